"""BoTorch-shaped model and acquisition objects over the gpx engine.

These mirror the reference's operator surface for the hot path so calling code reads like
``optimization/Bayesian*.py``:

  ExactGP(train_X, train_Y, params, outcome_transform=Standardize)   ≙ SingleTaskGP(train_X, train_Y, ...)
      .fit()                                                           ≙ building the exact posterior caches
      .posterior(X).mean / .variance                                   ≙ model.posterior(X) (Bayesian2.py:169-171)
  LogExpectedImprovement(model, best_f).sweep(X) -> (value, index)     ≙ analytic LogEI + raw-sample argmax
  ExpectedImprovement / UpperConfidenceBound / PosteriorVariance       ≙ the other analytic scores

Hyperparameters are either given (``params``) or fitted by maximum marginal likelihood with
``ExactGP.fit_hyperparameters`` (the fit_gpytorch_mll step of optimization/Bayesian.py:92-93,
objective and gradient on the GPU, L-BFGS-B on the host; see mll.py).  NOT_PD handling follows the reference's
jitter-retry policy (optimization/Bayesian6.py:481-488 through GPyTorch's psd_safe_cholesky, reference_jitter_schedule):
the factorisation is retried with the jitters of ``jitter_schedule`` before the NotPositiveDefiniteError propagates.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence

import torch

from ._capi import GPXTimeoutError, NotPositiveDefiniteError
from .engine import KERNEL_KINDS, GPEngine, GPState, KernelParams, botorch_default_lengthscale
from .transforms import Standardize


def reference_jitter_schedule(jitter_val: float = 1e-4, retry: float = 1e-2, max_tries: int = 3) -> tuple:
    """The diagonal jitters the reference's exact fit tries, in order (optimization/Bayesian6.py:482-488): GPyTorch's
    psd_safe_cholesky [upstream] first factors without jitter, then adds cholesky_jitter x 10^i for i < max_tries
    (settings.cholesky_max_tries = 3); the fit runs under cholesky_jitter(jitter_val = 1e-4, Bayesian6.py:66) and, if it
    still fails, again under cholesky_jitter(1e-2).  The union in order: 0, 1e-4, 1e-3, 1e-2, 1e-1, 1."""
    seq = [0.0]
    for base in (jitter_val, retry):
        for i in range(max_tries):
            j = base * 10.0 ** i
            if all(abs(j - s) > 1e-12 * j for s in seq):
                seq.append(j)
    return tuple(seq)


@dataclass
class Posterior:
    mean: torch.Tensor       # (m, T) untransformed
    variance: torch.Tensor   # (m, T) untransformed (all outputs share the kernel: identical columns scaled)


class ExactGP:
    """Exact GP with up to 8 outputs sharing X and the covariance (one factorisation, T right-hand sides)."""

    def __init__(self, train_X, train_Y, params: Optional[KernelParams] = None,
                 outcome_transform: Optional[Standardize] = None, engine=None,
                 jitter_schedule: Optional[Sequence[float]] = None, capacity: int = 0):
        self.engine = engine if engine is not None else GPEngine()
        dev = getattr(self.engine, "device", None)
        X = torch.as_tensor(train_X, dtype=torch.float64)
        Y = torch.as_tensor(train_Y, dtype=torch.float64)
        if Y.dim() == 1:
            Y = Y.unsqueeze(-1)
        if dev is not None:
            X, Y = X.to(dev), Y.to(dev)
        self.train_X, self.train_Y = X, Y
        d = X.shape[1]
        self.params = params or KernelParams("rbf", botorch_default_lengthscale(d), noise=1e-4)
        self.outcome_transform = outcome_transform
        self.jitter_schedule = tuple(jitter_schedule) if jitter_schedule is not None else reference_jitter_schedule()
        self.capacity = int(capacity)  # training points the factor's buffers reserve room for (later appends)
        self.state: Optional[GPState] = None
        self.jitter_used = None
        self.mll_result = None
        self.timeout_fallbacks = 0  # fits that fell back to the hand-off-free inverse path (see fit)

    @property
    def num_outputs(self) -> int:
        return self.train_Y.shape[1]

    @property
    def lengthscale(self):
        return self.params.lengthscales(self.train_X.shape[1])

    def _fit_once(self, Y, jit: float, inverse: bool):
        cap = self.capacity if self.capacity > self.train_X.shape[0] else 0
        return self.engine.fit(self.train_X, Y, self.params.replace(jitter=jit), capacity=cap, inverse=inverse)

    def fit(self) -> "ExactGP":
        """Gram + Cholesky + alpha with the reference's jitter retry (NotPositiveDefiniteError -> next jitter,
        optimization/Bayesian6.py:481-488).  The default update solves for alpha with one persistent launch whose
        workgroups hand blocks to each other; if that hand-off times out (GPXTimeoutError: its workgroups could not all
        become resident, e.g. beside a long kernel on another stream) the same jitter is refitted once through the
        hand-off-free path (W = L^{-T} by multi-launch TRTRI, alpha = W W^T y), so a BO run never ends on a timeout -
        the reference's fit has no such failure mode.  ``timeout_fallbacks`` counts those refits."""
        Y = self.train_Y
        if self.outcome_transform is not None:
            Y = self.outcome_transform.fit(Y).transform(Y)
        last = None
        for jit in self.jitter_schedule:
            try:
                try:
                    self.state = self._fit_once(Y, jit, inverse=False)
                except GPXTimeoutError:
                    self.timeout_fallbacks += 1
                    self.state = self._fit_once(Y, jit, inverse=True)
                self.jitter_used = jit
                return self
            except NotPositiveDefiniteError as e:  # reference: retry with larger cholesky_jitter
                last = e
        raise last

    def fit_hyperparameters(self, prior_set: str = "dim_scaled", fit_mean: bool = True,
                            options: Optional[dict] = None) -> "ExactGP":
        """Maximum marginal likelihood over the hyperparameters (all outputs share them), then refit the posterior
        caches at the optimum.  ``prior_set``: "dim_scaled" (BoTorch >= 0.12 SingleTaskGP), "gamma" (older
        BoTorch) or "none" (see mll.py)."""
        from .mll import fit_hyperparameters

        Y = self.train_Y
        if self.outcome_transform is not None:
            Y = self.outcome_transform.fit(Y).transform(Y)
        kind = self.params.kind if isinstance(self.params.kind, str) else \
            {v: k for k, v in KERNEL_KINDS.items()}[int(self.params.kind)]
        res = fit_hyperparameters(self.engine, self.train_X, Y, kind, prior_set, base=self.params, fit_mean=fit_mean,
                                  options=options)
        self.params = res.params
        self.mll_result = res
        return self.fit()

    def append_observations(self, X_new, Y_new) -> "ExactGP":
        """Add observations and update the posterior incrementally: the bordered Cholesky of the new
        rows (GPEngine.append, O(n^2 q)) instead of the full refit the reference runs after appending
        (optimization/Bayesian.py:163-174 then :89-94 next round; optimization/Bayesian7.py:628-631,639).  Valid
        because K depends only on the inputs and the (unchanged) hyperparameters; the outcome transform is refitted on
        all targets and alpha recomputed.  Falls back to ``fit`` (with the jitter schedule) when there is no state yet
        or the update is not positive definite."""
        dev = self.train_X.device
        X_new = torch.as_tensor(X_new, dtype=torch.float64).to(dev)
        Y_new = torch.as_tensor(Y_new, dtype=torch.float64).to(dev)
        if Y_new.dim() == 1:
            Y_new = Y_new.unsqueeze(-1)
        self.train_X = torch.cat([self.train_X, X_new.reshape(-1, self.train_X.shape[1])])
        self.train_Y = torch.cat([self.train_Y, Y_new.reshape(-1, self.train_Y.shape[1])])
        if self.state is None or self.state.n >= self.train_X.shape[0]:
            return self.fit()
        Y = self.train_Y
        if self.outcome_transform is not None:
            Y = self.outcome_transform.fit(Y).transform(Y)
        try:
            self.state = self.engine.append(self.state, self.train_X, Y)
        except NotPositiveDefiniteError:
            self.state = None
            return self.fit()
        return self

    def _untransform(self):
        ot = self.outcome_transform
        if ot is None:
            return None, None
        return [float(v) for v in ot.mean.reshape(-1)], [float(v) for v in ot.std.reshape(-1)]

    def posterior(self, X) -> Posterior:
        if self.state is None:
            self.fit()
        ym, ys = self._untransform()
        mean, var = self.engine.posterior(self.state, X, ym, ys)
        # variance of output t = var_std * s_t^2 (the engine returns output 0's scaling)
        if ys is not None:
            s = torch.tensor(ys, dtype=torch.float64, device=var.device)
            var_all = (var / (s[0] * s[0])).unsqueeze(-1) * (s * s)
            var_all = torch.clamp(var_all, min=1e-12)
        else:
            var_all = var.unsqueeze(-1).expand(-1, self.num_outputs).clone()
        return Posterior(mean=mean, variance=var_all)


class _Analytic:
    kind = "logei"

    def __init__(self, model: ExactGP, best_f: float = 0.0, beta: float = 4.0, output: int = 0,
                 weights: Optional[Sequence[float]] = None):
        self.model = model
        self.best_f = float(best_f)
        self.beta = float(beta)
        self.output = output
        self.weights = weights

    def _objective(self):
        """(alpha vector, y_mean, y_scale) of the scored output, in the engine's standardized space."""
        m = self.model
        if m.state is None:
            m.fit()
        ym, ys = m._untransform()
        if self.weights is not None:
            raise NotImplementedError("weighted objectives: combine alpha columns before sweeping")
        alpha = m.state.alpha[:, self.output]
        if ym is None:
            return alpha, 0.0, 1.0
        return alpha, ym[self.output], ys[self.output]

    def sweep(self, X, index_offset: int = 0, return_scores: bool = False):
        alpha, ym, ys = self._objective()
        return self.model.engine.acquire(self.model.state, X, self.kind, best_f=self.best_f, beta=self.beta,
                                         y_mean=ym, y_scale=ys, alpha=alpha, index_offset=index_offset,
                                         return_scores=return_scores)

    def __call__(self, X) -> torch.Tensor:
        return self.sweep(X, return_scores=True)[2]


class ExpectedImprovement(_Analytic):
    kind = "ei"


class LogExpectedImprovement(_Analytic):
    kind = "logei"


class UpperConfidenceBound(_Analytic):
    kind = "ucb"


class PosteriorVariance(_Analytic):
    kind = "variance"
