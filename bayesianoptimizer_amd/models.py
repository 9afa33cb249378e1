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
from typing import List, Optional, Sequence

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
    variance: torch.Tensor   # (m, T) untransformed


class ExactGP:
    """Exact GP with up to 8 outputs on one X.

    Shared mode (``params`` one KernelParams): the outputs share the covariance, noise and constant mean — ONE
    factorisation with T right-hand sides (the arithmetic is exact when the hyperparameters are tied).
    Independent mode (``params`` a sequence of T KernelParams, or ``independent_outputs=True``): T independent GPs, each
    with its own lengthscales, outputscale, noise and constant mean — BoTorch's multi-output SingleTaskGP
    (optimization/Bayesian1.py:108-116, SingleTaskGP(X, Y[n, 8], Standardize(m=8)): a batch of 8 independent GPs on one
    X [upstream]); fitted in one batched call (GPEngine.fit_outputs), hyperparameters by one L-BFGS-B over the
    concatenated vector (``fit_hyperparameters``: the sum of the per-output losses, as fit_gpytorch_mll minimises for a
    batched model [upstream])."""

    def __init__(self, train_X, train_Y, params=None, outcome_transform: Optional[Standardize] = None, engine=None,
                 jitter_schedule: Optional[Sequence[float]] = None, capacity: int = 0,
                 independent_outputs: Optional[bool] = None):
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
        T = Y.shape[1]
        base = KernelParams("rbf", botorch_default_lengthscale(d), noise=1e-4)
        if params is not None and not isinstance(params, KernelParams):
            params = list(params)
            if len(params) != T:
                raise ValueError(f"expected {T} kernel parameter sets (one per output), got {len(params)}")
            if independent_outputs is False:
                raise ValueError("a parameter set per output needs independent_outputs")
            independent_outputs = True
        self.independent = bool(independent_outputs)
        if self.independent and not isinstance(params, list):
            params = [(params or base).replace() for _ in range(T)]
        self.params = params if params is not None else base
        self.outcome_transform = outcome_transform
        self.jitter_schedule = tuple(jitter_schedule) if jitter_schedule is not None else reference_jitter_schedule()
        self.capacity = int(capacity)  # training points the factor's buffers reserve room for (later appends)
        self.state: Optional[GPState] = None          # shared mode
        self.states: Optional[List[GPState]] = None   # independent mode: one per output
        self.jitter_used = None       # shared: the jitter of the fit; independent: one per output
        self.pivot_failures = []      # (output or None, jitter, 0-based failing pivot) of every NOT_PD attempt
        self.mll_result = None
        self.timeout_fallbacks = 0  # fits that fell back to the hand-off-free inverse path (see fit)

    @property
    def num_outputs(self) -> int:
        return self.train_Y.shape[1]

    @property
    def fitted(self) -> bool:
        return (self.states if self.independent else self.state) is not None

    def output_params(self, t: int) -> KernelParams:
        return self.params[t] if self.independent else self.params

    @property
    def lengthscale(self):
        return self.output_params(0).lengthscales(self.train_X.shape[1])

    def _targets(self):
        Y = self.train_Y
        if self.outcome_transform is not None:
            Y = self.outcome_transform.fit(Y).transform(Y)
        return Y

    def _fit_once(self, Y, jit: float, inverse: bool):
        cap = self.capacity if self.capacity > self.train_X.shape[0] else 0
        return self.engine.fit(self.train_X, Y, self.params.replace(jitter=jit), capacity=cap, inverse=inverse)

    def fit(self) -> "ExactGP":
        """Gram + Cholesky + alpha with the reference's jitter retry (NotPositiveDefiniteError -> next jitter,
        optimization/Bayesian6.py:481-488).  The default update solves for alpha with one persistent launch whose
        workgroups hand blocks to each other; if that hand-off times out (GPXTimeoutError: its workgroups could not all
        become resident, e.g. beside a long kernel on another stream) the same jitter is refitted once through the
        hand-off-free path (W = L^{-T} by multi-launch TRTRI, alpha = W W^T y), so a BO run never ends on a timeout -
        the reference's fit has no such failure mode.  ``timeout_fallbacks`` counts those refits; ``pivot_failures``
        records every failed attempt's (output, jitter, pivot)."""
        Y = self._targets()
        self.pivot_failures = []
        if self.independent:
            return self._fit_outputs(Y)
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
                self.pivot_failures.append((None, jit, e.pivot))
                last = e
        raise last

    def _fit_outputs(self, Y) -> "ExactGP":
        """Independent mode: every output's fit in ONE batched call per attempt; an output whose factor fails moves to
        the next jitter of the schedule while the others keep theirs — psd_safe_cholesky adds jitter only to the
        failing members of a batch [upstream], so each output ends at the first jitter its own matrix accepts."""
        sched = self.jitter_schedule
        T = self.num_outputs
        level = [0] * T
        inverse = False
        prev = self.states
        while True:
            pj = [self.params[t].replace(jitter=sched[level[t]]) for t in range(T)]
            states = self.engine.fit_outputs(self.train_X, Y, pj, check=False, out=prev, inverse=inverse)
            info = self.engine.batch_info(states)
            if (info < 0).any() and not inverse:  # a timed-out hand-off: the hand-off-free path, same jitters
                self.timeout_fallbacks += 1
                inverse, prev = True, states
                continue
            bad = [t for t in range(T) if info[t] != 0]
            for t in bad:
                if info[t] < 0:
                    raise GPXTimeoutError(f"output {t}: in-launch hand-off timed out")
                self.pivot_failures.append((t, sched[level[t]], int(info[t]) - 1))
                level[t] += 1
                if level[t] >= len(sched):
                    raise NotPositiveDefiniteError(int(info[t]) - 1, f"output {t}: not positive definite at pivot "
                                                                     f"{int(info[t]) - 1} through the jitter schedule")
            if not bad:
                break
            prev = states
        self.states = states
        self.jitter_used = [sched[level[t]] for t in range(T)]
        return self

    def fit_hyperparameters(self, prior_set: str = "dim_scaled", fit_mean: bool = True,
                            options: Optional[dict] = None) -> "ExactGP":
        """Maximum marginal likelihood over the hyperparameters, then refit the posterior caches at the optimum.
        Shared mode: one parameter set for all outputs.  Independent mode: one set per output, all fitted by one
        L-BFGS-B over the concatenated vector on the sum of the per-output losses (mll.fit_hyperparameters_outputs).
        ``prior_set``: "dim_scaled" (BoTorch >= 0.12 SingleTaskGP), "gamma" (older BoTorch) or "none" (see mll.py)."""
        from .mll import fit_hyperparameters, fit_hyperparameters_outputs

        Y = self._targets()
        p0 = self.output_params(0)
        kind = p0.kind if isinstance(p0.kind, str) else {v: k for k, v in KERNEL_KINDS.items()}[int(p0.kind)]
        if self.independent:
            res = fit_hyperparameters_outputs(self.engine, self.train_X, Y, kind, prior_set, bases=self.params,
                                              fit_mean=fit_mean, options=options)
            self.params = list(res.params)
        else:
            res = fit_hyperparameters(self.engine, self.train_X, Y, kind, prior_set, base=self.params,
                                      fit_mean=fit_mean, options=options)
            self.params = res.params
        self.mll_result = res
        return self.fit()

    def append_observations(self, X_new, Y_new) -> "ExactGP":
        """Add observations and update the posterior incrementally: the bordered Cholesky of the new
        rows (GPEngine.append, O(n^2 q)) instead of the full refit the reference runs after appending
        (optimization/Bayesian.py:163-174 then :89-94 next round; optimization/Bayesian7.py:628-631,639).  Valid
        because K depends only on the inputs and the (unchanged) hyperparameters; the outcome transform is refitted on
        all targets and alpha recomputed.  Independent mode: each output's factor is bordered with its own parameters.
        Falls back to ``fit`` (with the jitter schedule) when there is no state yet or the update is not positive
        definite."""
        dev = self.train_X.device
        X_new = torch.as_tensor(X_new, dtype=torch.float64).to(dev)
        Y_new = torch.as_tensor(Y_new, dtype=torch.float64).to(dev)
        if Y_new.dim() == 1:
            Y_new = Y_new.unsqueeze(-1)
        self.train_X = torch.cat([self.train_X, X_new.reshape(-1, self.train_X.shape[1])])
        self.train_Y = torch.cat([self.train_Y, Y_new.reshape(-1, self.train_Y.shape[1])])
        n_fit = (self.states[0].n if self.states else 0) if self.independent else (self.state.n if self.state else 0)
        if not self.fitted or n_fit >= self.train_X.shape[0]:
            return self.fit()
        Y = self._targets()
        try:
            if self.independent:
                self.states = [self.engine.append(st, self.train_X, Y[:, t:t + 1])
                               for t, st in enumerate(self.states)]
            else:
                self.state = self.engine.append(self.state, self.train_X, Y)
        except NotPositiveDefiniteError:
            self.state = self.states = None
            return self.fit()
        return self

    def _untransform(self):
        ot = self.outcome_transform
        if ot is None:
            return None, None
        return [float(v) for v in ot.mean.reshape(-1)], [float(v) for v in ot.std.reshape(-1)]

    def posterior(self, X) -> Posterior:
        if not self.fitted:
            self.fit()
        ym, ys = self._untransform()
        if self.independent:
            cols_m, cols_v = [], []
            for t, st in enumerate(self.states):
                m_t, v_t = self.engine.posterior(st, X, None if ym is None else [ym[t]],
                                                 None if ys is None else [ys[t]])
                cols_m.append(m_t[:, 0])
                cols_v.append(v_t)
            return Posterior(mean=torch.stack(cols_m, 1), variance=torch.stack(cols_v, 1))
        mean, var = self.engine.posterior(self.state, X, ym, ys)
        # variance of output t = var_std * s_t^2 (the engine returns output 0's scaling)
        if ys is not None:
            s = torch.tensor(ys, dtype=torch.float64, device=var.device)
            var_all = (var / (s[0] * s[0])).unsqueeze(-1) * (s * s)
            var_all = torch.clamp(var_all, min=1e-12)
        else:
            var_all = var.unsqueeze(-1).expand(-1, self.num_outputs).clone()
        return Posterior(mean=mean, variance=var_all)

    def sweep_objective(self, X, kind: str, weights: Sequence[float], best_f: float = 0.0, beta: float = 4.0,
                        index_offset: int = 0, return_scores: bool = False):
        """Score the linear objective sum_t w_t f_t (f_t the untransformed outputs) over candidates X and reduce to
        (best value, lowest index among ties): independent mode through GPEngine.acquire_multi (the outputs'
        variances add), shared mode through one sweep with the combined alpha (the outputs share the posterior
        covariance: variance |w|^2 var)."""
        if not self.fitted:
            self.fit()
        ym, ys = self._untransform()
        T = self.num_outputs
        w = [float(v) for v in weights]
        if len(w) != T:
            raise ValueError(f"expected {T} objective weights, got {len(w)}")
        if self.independent:
            return self.engine.acquire_multi(self.states, X, kind, best_f=best_f, beta=beta, weights=w, y_mean=ym,
                                             y_scale=ys, index_offset=index_offset, return_scores=return_scores)
        st = self.state
        ymv = torch.zeros(T, dtype=torch.float64) if ym is None else torch.tensor(ym, dtype=torch.float64)
        ysv = torch.ones(T, dtype=torch.float64) if ys is None else torch.tensor(ys, dtype=torch.float64)
        wt = torch.tensor(w, dtype=torch.float64)
        # f = sum_t w_t (ym_t + ys_t (c + k*^T alpha_t)): scale s = |w * ys| (the shared standardised variance times s^2)
        ws = wt * ysv
        s = float(torch.linalg.vector_norm(ws))
        if s == 0.0:
            raise ValueError("objective weights are all zero")
        c = float(st.params.const_mean)
        alpha = (st.alpha[:, :T] @ ws.to(st.alpha.device)) / s
        y_mean = float((wt * ymv).sum()) + c * (float(ws.sum()) - s)
        return self.engine.acquire(st, X, kind, best_f=best_f, beta=beta, y_mean=y_mean, y_scale=s,
                                   alpha=alpha.contiguous(), index_offset=index_offset, return_scores=return_scores)


class _Analytic:
    kind = "logei"

    def __init__(self, model: ExactGP, best_f: float = 0.0, beta: float = 4.0, output: int = 0,
                 weights: Optional[Sequence[float]] = None):
        self.model = model
        self.best_f = float(best_f)
        self.beta = float(beta)
        self.output = output
        self.weights = weights

    def sweep(self, X, index_offset: int = 0, return_scores: bool = False):
        """Score candidates X on output ``output`` (or on the linear objective ``weights`` over all outputs, in
        untransformed units: ExactGP.sweep_objective) and reduce to (value, lowest index) on the device."""
        m = self.model
        if not m.fitted:
            m.fit()
        if self.weights is not None:
            return m.sweep_objective(X, self.kind, self.weights, best_f=self.best_f, beta=self.beta,
                                     index_offset=index_offset, return_scores=return_scores)
        ym, ys = m._untransform()
        t = self.output
        if m.independent:
            st, alpha = m.states[t], m.states[t].alpha[:, 0]
        else:
            st, alpha = m.state, m.state.alpha[:, t]
        return m.engine.acquire(st, X, self.kind, best_f=self.best_f, beta=self.beta,
                                y_mean=0.0 if ym is None else ym[t], y_scale=1.0 if ys is None else ys[t],
                                alpha=alpha, index_offset=index_offset, return_scores=return_scores)

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
