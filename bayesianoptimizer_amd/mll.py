"""Maximum-marginal-likelihood hyperparameter fit — the ``fit_gpytorch_mll`` step of the
reference (optimization/Bayesian.py:92-93, optimization/Bayesian1.py:114-115, optimization/Bayesian6.py:480-488).

Every objective evaluation runs on the GPU through the engine: Gram + Cholesky + L^{-T} + alpha
(``gpx_fit_f64``) and the fused K^{-1}-contraction gradient kernel (``gpx_mll_grad_f64``).  The host keeps only
what BoTorch/GPyTorch keep on the host [upstream]: the parameter transforms, the priors and scipy's L-BFGS-B.

Objective (ExactMarginalLogLikelihood [upstream], negated for minimisation):
    loss(raw) = ( -log p(y | theta) - sum_priors log prior(theta) ) / n,     theta = transform(raw)

Prior/constraint sets (the SingleTaskGP defaults differ by BoTorch version; the reference pins none):
  "dim_scaled"  BoTorch >= 0.12: RBF (or Matérn-5/2) ARD kernel without ScaleKernel;
                lengthscale LogNormal(sqrt2 + log(d)/2, sqrt3), constraint l >= 0.025 (no transform),
                initialised at the prior mode; noise LogNormal(-4, 1), constraint >= 1e-4 (no transform),
                initialised at the mode exp(-5); ConstantMean initialised at 0.
  "gamma"       BoTorch < 0.12: ScaleKernel(Matérn-5/2 ARD); lengthscale Gamma(3, 6) and outputscale Gamma(2, 0.15)
                through softplus (Positive), raw 0; noise Gamma(1.1, 0.05), constraint >= 1e-4 (no transform),
                initialised at the mode 2.0.
  "none"        no priors; softplus-positive lengthscale / outputscale / linear variances, noise >= 1e-4 through
                softplus (GaussianLikelihood default) — e.g. the ScaleKernel(Linear + Matérn-5/2) of
                optimization/Bayesian6.py:471-473.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import numpy as np

from ._capi import GPXError
from .engine import KernelParams

SQRT2 = math.sqrt(2.0)
SQRT3 = math.sqrt(3.0)
LOG_SQRT_2PI = 0.5 * math.log(2.0 * math.pi)


# ---- priors ----------------------------------------------------------------------------------------
@dataclass(frozen=True)
class LogNormalPrior:
    loc: float
    scale: float

    def log_prob(self, x: float) -> float:
        z = (math.log(x) - self.loc) / self.scale
        return -math.log(x) - math.log(self.scale) - LOG_SQRT_2PI - 0.5 * z * z

    def dlog_prob(self, x: float) -> float:
        return -1.0 / x - (math.log(x) - self.loc) / (self.scale * self.scale * x)

    @property
    def mode(self) -> float:
        return math.exp(self.loc - self.scale * self.scale)


@dataclass(frozen=True)
class GammaPrior:
    concentration: float
    rate: float

    def log_prob(self, x: float) -> float:
        a, b = self.concentration, self.rate
        return a * math.log(b) - math.lgamma(a) + (a - 1.0) * math.log(x) - b * x

    def dlog_prob(self, x: float) -> float:
        return (self.concentration - 1.0) / x - self.rate

    @property
    def mode(self) -> float:
        return max(self.concentration - 1.0, 0.0) / self.rate


# ---- transforms --------------------------------------------------------------------------------------
def _softplus(r: float) -> float:
    return r + math.log1p(math.exp(-r)) if r > 0 else math.log1p(math.exp(r))


def _softplus_inv(x: float) -> float:
    return x + math.log(-math.expm1(-x)) if x < 30 else x


def _sigmoid(r: float) -> float:
    return 1.0 / (1.0 + math.exp(-r)) if r >= 0 else math.exp(r) / (1.0 + math.exp(r))


@dataclass
class Hyper:
    """One scalar hyperparameter: natural value = lower + softplus(raw) (softplus) or raw (identity)."""

    name: str                    # "noise" | "const_mean" | "outputscale" | "lengthscale" | "linear_variance"
    index: Optional[int]         # dimension for ARD entries
    transform: str               # "identity" | "softplus"
    lower: Optional[float]       # constraint lower bound (natural units)
    prior: Optional[object]      # LogNormalPrior | GammaPrior | None
    init: float                  # natural initial value

    def to_natural(self, raw: float) -> float:
        if self.transform == "softplus":
            return (self.lower or 0.0) + _softplus(raw)
        return raw

    def to_raw(self, nat: float) -> float:
        if self.transform == "softplus":
            return _softplus_inv(max(nat - (self.lower or 0.0), 1e-300))
        return nat

    def dnat_draw(self, raw: float) -> float:
        return _sigmoid(raw) if self.transform == "softplus" else 1.0

    def raw_bounds(self):
        if self.transform == "identity" and self.lower is not None:
            return (self.lower, None)
        return (None, None)


@dataclass
class HyperSpec:
    kind: str
    d: int
    hypers: List[Hyper]
    base: KernelParams                       # values of the parameters that are not fitted

    def params_from_raw(self, raw: np.ndarray) -> KernelParams:
        p = self.base.replace()
        ls = list(p.lengthscales(self.d))
        lv = list(p.linear_variances(self.d))
        kw = {}
        for h, r in zip(self.hypers, raw):
            v = h.to_natural(float(r))
            if h.name == "lengthscale":
                ls[h.index] = v
            elif h.name == "linear_variance":
                lv[h.index] = v
            else:
                kw[h.name] = v
        return p.replace(lengthscale=ls, linear_variance=lv, **kw)

    def x0(self) -> np.ndarray:
        return np.array([h.to_raw(h.init) for h in self.hypers], dtype=np.float64)

    def bounds(self):
        return [h.raw_bounds() for h in self.hypers]


def default_spec(kind: str, d: int, prior_set: str = "dim_scaled", base: Optional[KernelParams] = None,
                 fit_mean: bool = True) -> HyperSpec:
    """The SingleTaskGP hyperparameters of the chosen BoTorch generation (module docstring)."""
    kind = kind.lower()
    hs: List[Hyper] = []
    if prior_set == "dim_scaled":
        lp = LogNormalPrior(SQRT2 + 0.5 * math.log(d), SQRT3)
        npr = LogNormalPrior(-4.0, 1.0)
        hs.append(Hyper("noise", None, "identity", 1e-4, npr, npr.mode))
        if fit_mean:
            hs.append(Hyper("const_mean", None, "identity", None, None, 0.0))
        hs += [Hyper("lengthscale", k, "identity", 2.5e-2, lp, lp.mode) for k in range(d)]
        outputscale = 1.0
    elif prior_set == "gamma":
        npr, opr, lpr = GammaPrior(1.1, 0.05), GammaPrior(2.0, 0.15), GammaPrior(3.0, 6.0)
        hs.append(Hyper("noise", None, "identity", 1e-4, npr, npr.mode))
        if fit_mean:
            hs.append(Hyper("const_mean", None, "identity", None, None, 0.0))
        hs.append(Hyper("outputscale", None, "softplus", 0.0, opr, _softplus(0.0)))
        hs += [Hyper("lengthscale", k, "softplus", 0.0, lpr, _softplus(0.0)) for k in range(d)]
        outputscale = _softplus(0.0)
    elif prior_set == "none":
        hs.append(Hyper("noise", None, "softplus", 1e-4, None, 1e-4 + _softplus(0.0)))
        if fit_mean:
            hs.append(Hyper("const_mean", None, "identity", None, None, 0.0))
        hs.append(Hyper("outputscale", None, "softplus", 0.0, None, _softplus(0.0)))
        hs += [Hyper("lengthscale", k, "softplus", 0.0, None, _softplus(0.0)) for k in range(d)]
        if kind == "scale_linear_matern52":
            hs += [Hyper("linear_variance", k, "softplus", 0.0, None, _softplus(0.0)) for k in range(d)]
        outputscale = _softplus(0.0)
    else:
        raise ValueError(f"unknown prior set '{prior_set}' (dim_scaled | gamma | none)")
    if base is None:
        base = KernelParams(kind, 1.0, outputscale=outputscale)
    spec = HyperSpec(kind=kind, d=d, hypers=hs, base=base.replace(kind=kind))
    # initial values of the fitted entries also seed ``base`` (used for anything not fitted)
    spec.base = spec.params_from_raw(spec.x0())
    return spec


# ---- objective -------------------------------------------------------------------------------------
def _feasible(spec: HyperSpec, raw) -> bool:
    """A line-search trial point outside the parameter domain (a softplus underflowing to 0, an overflow) scores +inf,
    so L-BFGS-B backtracks (GPyTorch's NaN loss plays that role in fit_gpytorch_mll_scipy [upstream])."""
    nat = [h.to_natural(float(r)) for h, r in zip(spec.hypers, raw)]
    return all(np.isfinite(v) for v in nat) and not any(v <= 0.0 for h, v in zip(spec.hypers, nat)
                                                        if h.name in ("lengthscale", "outputscale", "noise"))


def _loss_grad(spec: HyperSpec, raw, g: dict, n: int):
    """(loss, dloss/draw) of one output: (-log p(y) - sum_priors log prior) / n from the natural-parameter gradient
    dict ``g`` (ExactMarginalLogLikelihood's value divided by num_data [upstream])."""
    loss = g["nll"]
    grad = np.empty(len(spec.hypers))
    for i, (h, r) in enumerate(zip(spec.hypers, raw)):
        nat = h.to_natural(float(r))
        dn = g[h.name][h.index] if h.index is not None else g[h.name]
        if h.prior is not None:
            loss -= h.prior.log_prob(nat)
            dn = dn - h.prior.dlog_prob(nat)
        grad[i] = dn * h.dnat_draw(float(r))
    return loss / n, grad / n


def objective(spec: HyperSpec, value_grad: Callable, n: int):
    """loss(raw), dloss/draw with value_grad(params) -> dict of -log p(y) and its natural-parameter gradient
    (engine.mll_value_grad or the oracle's mll_value_grad)."""

    def f(raw):
        raw = np.asarray(raw, dtype=np.float64)
        if not _feasible(spec, raw):
            return np.inf, np.zeros_like(raw)
        try:
            g = value_grad(spec.params_from_raw(raw))
        except (GPXError, np.linalg.LinAlgError):  # indefinite through the jitter ladder: +inf, L-BFGS-B backtracks
            return np.inf, np.zeros_like(raw)
        if not np.isfinite(g["nll"]):
            return np.inf, np.zeros_like(raw)
        return _loss_grad(spec, raw, g, n)

    return f


def objective_outputs(specs: Sequence[HyperSpec], value_grad_all: Callable, n: int):
    """The multi-output loss over the concatenated raw vector [raw_0, raw_1, ...]: the sum of the per-output losses
    (BoTorch's fit_gpytorch_mll on a batched model sums the batch of ExactMarginalLogLikelihood values, each with its
    own prior terms [upstream]); value_grad_all(list of params) -> list of per-output dicts (one batched evaluation)."""
    sizes = [len(sp.hypers) for sp in specs]
    offs = np.concatenate([[0], np.cumsum(sizes)])

    def f(raw):
        raw = np.asarray(raw, dtype=np.float64)
        parts = [raw[offs[t]:offs[t + 1]] for t in range(len(specs))]
        if not all(_feasible(sp, r) for sp, r in zip(specs, parts)):
            return np.inf, np.zeros_like(raw)
        try:
            gs = value_grad_all([sp.params_from_raw(r) for sp, r in zip(specs, parts)])
        except (GPXError, np.linalg.LinAlgError):
            return np.inf, np.zeros_like(raw)
        if not all(np.isfinite(g["nll"]) for g in gs):
            return np.inf, np.zeros_like(raw)
        loss = 0.0
        grad = np.empty_like(raw)
        for t, (sp, r, g) in enumerate(zip(specs, parts, gs)):
            lt, gt = _loss_grad(sp, r, g, n)
            loss += lt
            grad[offs[t]:offs[t + 1]] = gt
        return loss, grad

    return f


@dataclass
class MLLFitResult:
    params: KernelParams
    loss: float                 # final (-mll) = (nll - log priors) / n
    nll: float                  # final -log p(y)
    n_evals: int
    success: bool
    message: str
    raw: np.ndarray = field(default_factory=lambda: np.zeros(0))


def fit_hyperparameters(engine, X, y, kind: str = "rbf", prior_set: str = "dim_scaled",
                        base: Optional[KernelParams] = None, fit_mean: bool = True,
                        options: Optional[dict] = None, value_grad: Optional[Callable] = None,
                        x0: Optional[Sequence[float]] = None) -> MLLFitResult:
    """L-BFGS-B over the raw hyperparameters, like fit_gpytorch_mll -> fit_gpytorch_mll_scipy [upstream].

    ``engine`` provides ``mll_value_grad(X, y, params)`` (GPEngine: GPU; tests inject the oracle through
    ``value_grad``).  ``options`` go to scipy.optimize.minimize (scipy's L-BFGS-B defaults otherwise).
    """
    from scipy.optimize import minimize

    Xn = np.asarray(X.cpu() if hasattr(X, "cpu") else X, dtype=np.float64)
    yn = np.asarray(y.cpu() if hasattr(y, "cpu") else y, dtype=np.float64)
    yn = yn.reshape(-1, 1) if yn.ndim == 1 else yn  # T columns share the hyperparameters
    n, d = Xn.shape
    spec = default_spec(kind, d, prior_set, base, fit_mean)
    if value_grad is None:
        state = [None]

        def value_grad(p):
            res, state[0] = engine.mll_value_grad(X, y, p, state=state[0])
            return res

    f = objective(spec, value_grad, n)
    last = {}

    def fg(raw):
        v, g = f(raw)
        last["v"] = v
        return v, g

    start = spec.x0() if x0 is None else np.asarray(x0, dtype=np.float64)
    res = minimize(fg, start, jac=True, method="L-BFGS-B", bounds=spec.bounds(), options=options or {})
    p = spec.params_from_raw(res.x)
    final = value_grad(p)
    loss, _ = f(res.x)
    return MLLFitResult(params=p, loss=float(loss), nll=float(final["nll"]), n_evals=int(res.nfev),
                        success=bool(res.success), message=str(res.message), raw=res.x.copy())


@dataclass
class MLLFitOutputsResult:
    params: List[KernelParams]  # one per output
    loss: float                 # final sum over outputs of (-mll_t)
    nll: List[float]            # final -log p(y_t) per output
    n_evals: int
    success: bool
    message: str
    raw: np.ndarray = field(default_factory=lambda: np.zeros(0))


def fit_hyperparameters_outputs(engine, X, Y, kind: str = "rbf", prior_set: str = "dim_scaled",
                                bases: Optional[Sequence[KernelParams]] = None, fit_mean: bool = True,
                                options: Optional[dict] = None, value_grad_all: Optional[Callable] = None,
                                x0: Optional[Sequence[float]] = None) -> MLLFitOutputsResult:
    """Hyperparameters of T independent outputs on one X (Y: n x T), each output its own set — the multi-output
    SingleTaskGP's fit_gpytorch_mll (optimization/Bayesian1.py:114-115 [upstream]): ONE L-BFGS-B over the concatenated
    raw vector on the summed loss.  Every evaluation is one batched fit of all outputs and one batched gradient
    (GPEngine.mll_value_grad_outputs); tests inject the oracle through ``value_grad_all``."""
    from scipy.optimize import minimize

    Xn = np.asarray(X.cpu() if hasattr(X, "cpu") else X, dtype=np.float64)
    Yn = np.asarray(Y.cpu() if hasattr(Y, "cpu") else Y, dtype=np.float64)
    Yn = Yn.reshape(-1, 1) if Yn.ndim == 1 else Yn
    n, d = Xn.shape
    T = Yn.shape[1]
    bases = list(bases) if bases is not None else [None] * T
    if len(bases) != T:
        raise ValueError(f"expected {T} base parameter sets, got {len(bases)}")
    specs = [default_spec(kind, d, prior_set, bases[t], fit_mean) for t in range(T)]
    if value_grad_all is None:
        state = [None]

        def value_grad_all(ps):
            res, state[0] = engine.mll_value_grad_outputs(X, Y, ps, states=state[0])
            return res

    f = objective_outputs(specs, value_grad_all, n)
    start = np.concatenate([sp.x0() for sp in specs]) if x0 is None else np.asarray(x0, dtype=np.float64)
    bounds = [b for sp in specs for b in sp.bounds()]
    res = minimize(f, start, jac=True, method="L-BFGS-B", bounds=bounds, options=options or {})
    sizes = np.concatenate([[0], np.cumsum([len(sp.hypers) for sp in specs])])
    ps = [sp.params_from_raw(res.x[sizes[t]:sizes[t + 1]]) for t, sp in enumerate(specs)]
    final = value_grad_all(ps)
    loss, _ = f(res.x)
    return MLLFitOutputsResult(params=ps, loss=float(loss), nll=[float(g["nll"]) for g in final],
                               n_evals=int(res.nfev), success=bool(res.success), message=str(res.message),
                               raw=res.x.copy())
