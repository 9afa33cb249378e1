"""Gradient-based acquisition optimisation over the GPU posterior.

The reference picks its next batch with BoTorch's ``optimize_acqf`` on a q-batch MC ``qLogExpectedImprovement``:
``optimization/Bayesian.py:96-113`` (q = batch_size, num_restarts 10, raw_samples 1024, 512 Sobol base samples,
options {"batch_limit": 5, "maxiter": 200}) and ``optimization/Bayesian2.py:218-245`` (LinearMCObjective over the 8
outputs, 256 base samples, num_restarts 8, raw_samples 256).  This module mirrors that surface [upstream: BoTorch
``optimize_acqf`` / ``gen_batch_initial_conditions`` / ``initialize_q_batch`` / ``gen_candidates_scipy``,
``qLogExpectedImprovement``, ``SobolQMCNormalSampler``, ``LinearMCObjective``]:

* the O(n^2 q) posterior work — q-batch means, covariances and their derivatives w.r.t. the candidates — runs in
  libgpx.so (``gpx_moments_grad_f64``: K* on the device, K^{-1} K* = W (W^T K*) on fp64 MFMA, fused first-argument
  kernel derivatives), wrapped as a torch autograd Function so the small q x q Monte-Carlo part differentiates with
  torch on the same device (BoTorch differentiates the whole posterior with autograd);
* the host keeps what BoTorch keeps on the host: scipy's L-BFGS-B over the flattened restarts.

Parity definition (parity unpinned: BoTorch is not installed and has no fixtures here): qLogEI follows
BoTorch's log-space form — log-improvement with the fat-tailed softplus (softplus + 0.1 * Cauchy, tau_relu = 1e-6) or
the plain log-softplus (``fat=False``), q-reduction by the smooth max tau_max * logsumexp(x / tau_max) (tau_max =
1e-2; BoTorch's fat q-reduction tail is not restated — identical for q = 1), sample reduction logmeanexp.  Base
samples are scrambled Sobol points (``torch.quasirandom.SobolEngine``) mapped through the inverse normal cdf.
oracle/gp_oracle.py restates the same definitions in NumPy for the tests.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import numpy as np
import torch

from . import _capi

TAU_RELU = 1e-6
TAU_MAX = 1e-2
_LOG_SQRT_2PI = 0.5 * math.log(2.0 * math.pi)
_LOG_SQRT_PI_DIV_2 = 0.5 * math.log(math.pi / 2.0)
_INV_SQRT_2 = 1.0 / math.sqrt(2.0)
_NEG_INV_SQRT_EPS = -1.0 / math.sqrt(np.finfo(np.float64).eps)
GPYTORCH_MIN_VAR_F64 = 1e-10
BOTORCH_MIN_VAR = 1e-12


# ---- posterior moments with gradients (GPU) -----------------------------------------------------------------------
class _Moments(torch.autograd.Function):
    """(mean (m,), cov (m, q)) of consecutive q-batches of candidates; backward from gpx_moments_grad_f64's
    derivatives: dL/dx_aj = gmean[a] dmean[a, j] + sum_c (G[a, c] + G[c, a]) dcov[a, j, c]."""

    @staticmethod
    def forward(ctx, Xs, engine, state, q, alpha):
        mean, dmean, cov, dcov = engine.moments_grad(state, Xs.detach(), q, alpha)
        ctx.save_for_backward(dmean, dcov)
        ctx.q = q
        return mean, cov

    @staticmethod
    def backward(ctx, gmean, gcov):
        dmean, dcov = ctx.saved_tensors
        q = ctx.q
        m, d = dmean.shape
        gX = torch.zeros_like(dmean)
        if gmean is not None:
            gX = gX + gmean.unsqueeze(-1) * dmean
        if gcov is not None:
            G = gcov.reshape(m // q, q, q)
            Gs = G + G.transpose(1, 2)
            gX = gX + torch.einsum("bac,bajc->baj", Gs, dcov.reshape(m // q, q, d, q)).reshape(m, d)
        return gX, None, None, None, None


class _Objective:
    """Scalar objective of the model's outputs in original units: a linear combination (LinearMCObjective,
    Bayesian2.py:213-214) or one output, as a sum of Gaussian terms (state, alpha, mean scale, variance scale) plus an
    offset.  Shared covariance (one factorisation): ONE term, the objective's mean sum_t w_t (y_mean_t + s_t mu_t) from
    the combined alpha and its covariance (sum_t w_t^2 s_t^2) Sigma_std.  Independent outputs (ExactGP independent
    mode, the multi-output SingleTaskGP): one term per output with a non-zero weight — mean sum_t w_t s_t mu_t + sum_t
    w_t y_mean_t, covariance sum_t w_t^2 s_t^2 Sigma_t (the outputs are independent a posteriori)."""

    def __init__(self, model, weights: Optional[Sequence[float]] = None, output: int = 0):
        T = model.num_outputs
        w = torch.zeros(T, dtype=torch.float64)
        if weights is not None:
            w = torch.as_tensor(weights, dtype=torch.float64).reshape(-1)
            if w.numel() != T:
                raise ValueError(f"expected {T} objective weights, got {w.numel()}")
        else:
            w[output] = 1.0
        ym, ys = model._untransform()
        ym = torch.tensor(ym if ym is not None else [0.0] * T, dtype=torch.float64)
        ys = torch.tensor(ys if ys is not None else [1.0] * T, dtype=torch.float64)
        ws = w * ys
        self.terms = []
        if getattr(model, "independent", False):
            for t in range(T):
                if float(ws[t]) != 0.0:
                    st = model.states[t]
                    self.terms.append((st, st.alpha[:, 0].contiguous(), float(ws[t]), float(ws[t]) ** 2))
            self.offset = float((w * ym).sum())
            self.var_scale = float((ws * ws).sum())
            return
        st = model.state
        dev = st.alpha.device
        alpha = (st.alpha * ws.to(dev).unsqueeze(0)).sum(dim=1).contiguous()
        cm = float(st.params.const_mean)
        self.offset = float((w * ym).sum()) + cm * (float(ws.sum()) - 1.0)
        self.var_scale = float((ws * ws).sum())
        self.terms.append((st, alpha, 1.0, self.var_scale))


def posterior_moments(model, X: torch.Tensor, objective: Optional[_Objective] = None, floor_terms: bool = False):
    """Mean (B, q) and covariance (B, q, q) of the objective at X (B, q, d), differentiable w.r.t. X (noise-free
    posterior, like BoTorch's acquisition functions).  ``model``: a fitted models.ExactGP.  ``floor_terms`` (q = 1):
    each term's standardised variance floored at GPyTorch's 1e-10 before scaling, as the GPU sweep does."""
    obj = objective or _Objective(model)
    B, q, d = X.shape
    mean_t = torch.full((B, q), obj.offset, dtype=torch.float64, device=X.device)
    cov_t = torch.zeros((B, q, q), dtype=torch.float64, device=X.device)
    for st, alpha, ms, vs in obj.terms:
        mean, cov = _Moments.apply(X.reshape(B * q, d), model.engine, st, q, alpha)
        cov = cov.reshape(B, q, q)
        if floor_terms:
            cov = torch.clamp(cov, min=GPYTORCH_MIN_VAR_F64)
        mean_t = mean_t + ms * mean.reshape(B, q)
        cov_t = cov_t + vs * cov
    return mean_t, cov_t


# ---- smooth maths (BoTorch safe_math [upstream], restated) -----------------------------------------------------
def _phi(u):
    return torch.exp(-0.5 * u * u) / math.sqrt(2.0 * math.pi)


def _log1mexp(x):
    xs = torch.clamp(x, max=-1e-300)
    return torch.where(x > -math.log(2.0), torch.log(-torch.expm1(xs)), torch.log1p(-torch.exp(torch.clamp(x, max=0.0))))


def log_ei_helper(u):
    """log(phi(u) + u Phi(u)) with the two-branch form of the GPU finalize kernel (gpx_sweep.hip)."""
    uu = torch.clamp(u, min=-1.0)
    upper = torch.log(_phi(uu) + uu * torch.special.ndtr(uu))
    u_lo = torch.clamp(u, max=-1.0)
    u_eps = torch.clamp(u_lo, min=_NEG_INV_SQRT_EPS)
    w = torch.log(torch.special.erfcx(-u_eps * _INV_SQRT_2) * u_eps.abs()) + _LOG_SQRT_PI_DIV_2
    log_phi = -0.5 * u_lo * u_lo - _LOG_SQRT_2PI
    lower = log_phi + torch.where(u_lo > _NEG_INV_SQRT_EPS, _log1mexp(w), -2.0 * torch.log(u_lo.abs()))
    return torch.where(u > -1.0, upper, lower)


def log_softplus(x, tau: float = 1.0):
    y = x / tau
    ys = torch.clamp(y, min=-37.0)
    return math.log(tau) + torch.where(y > -37.0, torch.log(torch.nn.functional.softplus(ys)), y)


def log_fatplus(x, tau: float = 1.0):
    """log(tau * (softplus(x / tau) + 0.1 / (1 + (x / tau)^2))): BoTorch's fat-tailed ReLU approximation."""
    y = x / tau
    return math.log(tau) + torch.log(torch.nn.functional.softplus(y) + 0.1 / (1.0 + y * y))


def smooth_amax(x, tau: float, dim: int = -1):
    return tau * torch.logsumexp(x / tau, dim=dim)


def logmeanexp(x, dim: int = 0):
    return torch.logsumexp(x, dim=dim) - math.log(x.shape[dim])


# ---- samplers / objectives -------------------------------------------------------------------------------------
class SobolQMCNormalSampler:
    """Scrambled-Sobol N(0, 1) base samples (BoTorch SobolQMCNormalSampler / draw_sobol_normal_samples [upstream]):
    u from SobolEngine(dimension=q, scramble=True, seed), z = sqrt(2) erfinv(2 v - 1) with v = 0.5 + (1 - eps)(u - 0.5).
    Fixed per (q, seed): the same base samples at every L-BFGS-B evaluation (BoTorch fixes them too)."""

    def __init__(self, sample_shape=torch.Size([512]), seed: Optional[int] = None):
        self.sample_shape = torch.Size(sample_shape)
        self.seed = int(seed) if seed is not None else int(torch.randint(0, 1_000_000, (1,)).item())
        self._cache = {}

    def base_samples(self, q: int, device) -> torch.Tensor:
        key = (q, str(device))
        if key not in self._cache:
            n = int(np.prod(self.sample_shape))
            eng = torch.quasirandom.SobolEngine(dimension=q, scramble=True, seed=self.seed)
            u = eng.draw(n, dtype=torch.float64)
            eps = torch.finfo(torch.float64).eps
            v = 0.5 + (1.0 - eps) * (u - 0.5)
            self._cache[key] = (torch.erfinv(2.0 * v - 1.0) * math.sqrt(2.0)).to(device)
        return self._cache[key]


class LinearMCObjective:
    """Weighted sum of the model outputs (Bayesian2.py:213-214)."""

    def __init__(self, weights):
        self.weights = [float(w) for w in torch.as_tensor(weights).reshape(-1)]


def psd_safe_cholesky(S: torch.Tensor, max_tries: int = 3) -> torch.Tensor:
    """Batched Cholesky with GPyTorch's jitter retry (1e-8 for float64, x10 per try) [upstream]."""
    L, info = torch.linalg.cholesky_ex(S)
    if not bool((info > 0).any()):
        return L
    eye = torch.eye(S.shape[-1], dtype=S.dtype, device=S.device)
    jitter = 1e-8
    for _ in range(max_tries):
        L, info = torch.linalg.cholesky_ex(S + jitter * eye)
        if not bool((info > 0).any()):
            return L
        jitter *= 10.0
    raise torch.linalg.LinAlgError("q-batch posterior covariance not positive definite after jitter")


# ---- acquisition functions (differentiable in X of shape B x q x d) -----------------------------------------
class AnalyticAcquisition:
    """q = 1 analytic scores on the differentiable posterior: EI / LogEI / UCB / posterior variance (the forms of the
    GPU sweep, gpx_sweep.hip; variance floors of GPyTorch 1e-10 (standardised) and BoTorch 1e-12)."""

    kind = "logei"

    def __init__(self, model, best_f: float = 0.0, beta: float = 4.0, objective: Optional[LinearMCObjective] = None,
                 output: int = 0):
        self.model = model
        self.best_f = float(best_f)
        self.beta = float(beta)
        self.objective = _Objective(model, objective.weights if objective is not None else None, output)

    def __call__(self, X: torch.Tensor) -> torch.Tensor:
        if X.dim() == 2:
            X = X.unsqueeze(1)
        if X.shape[1] != 1:
            raise ValueError("analytic acquisition functions take q = 1 (X: B x 1 x d)")
        mu, cov = posterior_moments(self.model, X, self.objective, floor_terms=True)
        mu = mu[:, 0]
        var = torch.clamp(cov[:, 0, 0], min=BOTORCH_MIN_VAR)
        sigma = torch.sqrt(var)
        if self.kind == "variance":
            return var
        if self.kind == "ucb":
            return mu + math.sqrt(self.beta) * sigma
        u = (mu - self.best_f) / sigma
        if self.kind == "ei":
            return sigma * (_phi(u) + u * torch.special.ndtr(u))
        return log_ei_helper(u) + torch.log(sigma)


class LogExpectedImprovement(AnalyticAcquisition):
    kind = "logei"


class ExpectedImprovement(AnalyticAcquisition):
    kind = "ei"


class UpperConfidenceBound(AnalyticAcquisition):
    kind = "ucb"


class PosteriorVariance(AnalyticAcquisition):
    kind = "variance"


class qLogExpectedImprovement:
    """MC q-batch log expected improvement (the acquisition of Bayesian.py:100-101 and Bayesian2.py:226-231):
    samples f = mu + L z of the objective's joint q-batch posterior, log-improvement log_fatplus(f - best_f, tau_relu)
    (or log_softplus with fat=False), smooth max over q (tau_max), logmeanexp over the samples."""

    def __init__(self, model, best_f: float, sampler: Optional[SobolQMCNormalSampler] = None,
                 objective: Optional[LinearMCObjective] = None, fat: bool = True, tau_max: float = TAU_MAX,
                 tau_relu: float = TAU_RELU, output: int = 0):
        self.model = model
        self.best_f = float(best_f)
        self.sampler = sampler or SobolQMCNormalSampler(torch.Size([512]))
        self.objective = _Objective(model, objective.weights if objective is not None else None, output)
        self.fat = fat
        self.tau_max = float(tau_max)
        self.tau_relu = float(tau_relu)

    def __call__(self, X: torch.Tensor) -> torch.Tensor:
        if X.dim() == 2:
            X = X.unsqueeze(0)
        q = X.shape[1]
        mu, cov = posterior_moments(self.model, X, self.objective)
        z = self.sampler.base_samples(q, X.device)
        return qlogei_from_moments(mu, cov, z, self.best_f, self.fat, self.tau_max, self.tau_relu)


def qlogei_from_moments(mu: torch.Tensor, cov: torch.Tensor, z: torch.Tensor, best_f: float, fat: bool = True,
                        tau_max: float = TAU_MAX, tau_relu: float = TAU_RELU) -> torch.Tensor:
    """qLogEI of q-batches from their joint posterior: mu (B, q), cov (B, q, q), base samples z (S, q) -> (B,)."""
    cov = 0.5 * (cov + cov.transpose(1, 2))
    L = psd_safe_cholesky(cov)
    f = mu.unsqueeze(0) + torch.einsum("bij,sj->sbi", L, z)  # S x B x q
    li = log_fatplus(f - best_f, tau_relu) if fat else log_softplus(f - best_f, tau_relu)
    return logmeanexp(smooth_amax(li, tau_max, dim=-1), dim=0)


# ---- optimize_acqf ------------------------------------------------------------------------------------------------
def initialize_q_batch(X: torch.Tensor, Y: torch.Tensor, n: int, eta: float = 1.0,
                       generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """Boltzmann sampling of n restart points from raw samples X (N x q x d) with acquisition values Y (N), the
    best raw sample always included (BoTorch initialize_q_batch [upstream])."""
    N = X.shape[0]
    if n > N:
        raise ValueError(f"n ({n}) cannot exceed the number of raw samples ({N})")
    if n == N:
        return X
    Yc = Y.detach().cpu()
    Ystd = Yc.std()
    if not torch.isfinite(Ystd) or Ystd == 0:
        return X[torch.randperm(N, generator=generator)[:n].to(X.device)]
    max_idx = int(torch.argmax(Yc))
    etaZ = eta * (Yc - Yc.mean()) / Ystd
    weights = torch.exp(etaZ)
    while torch.isinf(weights).any():
        etaZ = etaZ * 0.5
        weights = torch.exp(etaZ)
    idcs = torch.multinomial(weights, n, replacement=False, generator=generator)
    if max_idx not in idcs.tolist():
        idcs[-1] = max_idx
    return X[idcs.to(X.device)]


def _eval_batched(acq, X: torch.Tensor, chunk: int) -> torch.Tensor:
    with torch.no_grad():
        return torch.cat([acq(X[s:s + chunk]) for s in range(0, X.shape[0], chunk)])


def gen_batch_initial_conditions(acq, bounds: torch.Tensor, q: int, num_restarts: int, raw_samples: int,
                                 seed: Optional[int] = None, eta: float = 1.0) -> torch.Tensor:
    """raw_samples scrambled-Sobol q-batches in the bounds, scored on the GPU posterior, then initialize_q_batch."""
    d = bounds.shape[1]
    seed = int(seed) if seed is not None else int(torch.randint(0, 1_000_000, (1,)).item())
    u = torch.quasirandom.SobolEngine(dimension=q * d, scramble=True, seed=seed).draw(raw_samples, dtype=torch.float64)
    lo, hi = bounds[0].to(torch.float64), bounds[1].to(torch.float64)
    X = (lo + (hi - lo) * u.view(raw_samples, q, d).to(bounds.device)).contiguous()
    max_m = _capi.GPX_MAX_GRAD_CANDIDATES // q
    Y = _eval_batched(acq, X, max(1, min(max_m, 2048 // q if q <= 2048 else 1)))
    g = torch.Generator().manual_seed(seed)
    return initialize_q_batch(X, Y, num_restarts, eta=eta, generator=g)


def gen_candidates_scipy(X0: torch.Tensor, acq, lower: torch.Tensor, upper: torch.Tensor, maxiter: int = 200):
    """L-BFGS-B (scipy, host) on the flattened restarts, jointly minimising -sum(acq) like BoTorch's
    gen_candidates_scipy [upstream]; every objective/gradient evaluation is one GPU posterior-gradient call."""
    from scipy.optimize import minimize

    shape = X0.shape
    dev = X0.device
    lo = lower.expand(shape).reshape(-1).cpu().numpy()
    hi = upper.expand(shape).reshape(-1).cpu().numpy()

    def f_and_g(x):
        X = torch.tensor(x, dtype=torch.float64, device=dev).view(shape).requires_grad_(True)
        loss = -acq(X).sum()
        (g,) = torch.autograd.grad(loss, X)
        gn = g.detach().cpu().numpy().ravel()
        val = float(loss.item())
        if not np.isfinite(val):
            return np.inf, np.zeros_like(gn)
        return val, np.nan_to_num(gn)

    x0 = X0.detach().cpu().numpy().ravel()
    res = minimize(f_and_g, x0, jac=True, method="L-BFGS-B", bounds=list(zip(lo, hi)),
                   options={"maxiter": int(maxiter)})
    X = torch.tensor(np.clip(res.x, lo, hi), dtype=torch.float64, device=dev).view(shape)
    with torch.no_grad():
        vals = acq(X)
        # the joint objective is a sum: a restart may give up value for another's gain; keep its better end point
        v0 = acq(X0.detach())
        worse = ~(vals >= v0)
        if bool(worse.any()):
            X = torch.where(worse.view(-1, 1, 1), X0.detach(), X)
            vals = torch.where(worse, v0, vals)
    return X, vals


def optimize_acqf(acq_function, bounds, q: int, num_restarts: int, raw_samples: int, options: Optional[dict] = None,
                  return_best_only: bool = True, seed: Optional[int] = None):
    """BoTorch-shaped optimize_acqf (Bayesian.py:105-112, Bayesian2.py:240-245): raw-sample initialisation, restarts
    in batches of ``batch_limit`` refined with L-BFGS-B (``maxiter``), best restart returned as (q x d, value)."""
    options = dict(options or {})
    dev = acq_function.model.engine.device
    bounds = torch.as_tensor(bounds, dtype=torch.float64, device=dev)
    if bounds.dim() != 2 or bounds.shape[0] != 2:
        raise ValueError("bounds must be 2 x d")
    if q < 1 or q > _capi.GPX_MAX_Q:
        raise ValueError(f"q must be in [1, {_capi.GPX_MAX_Q}]")
    X0 = gen_batch_initial_conditions(acq_function, bounds, q, num_restarts, raw_samples, seed=seed,
                                      eta=float(options.get("eta", 1.0)))
    batch_limit = int(options.get("batch_limit", num_restarts))
    maxiter = int(options.get("maxiter", 200))
    Xs, vs = [], []
    for s in range(0, X0.shape[0], batch_limit):
        X, v = gen_candidates_scipy(X0[s:s + batch_limit], acq_function, bounds[0], bounds[1], maxiter)
        Xs.append(X)
        vs.append(v)
    X = torch.cat(Xs)
    v = torch.cat(vs)
    if not return_best_only:
        return X, v
    b = int(torch.argmax(v))
    return X[b], v[b]
