"""Test-only stand-in for GPEngine backed by the CPU oracle.

Used by the CPU plumbing tests (BASELINE configs[0]: the drop-in driven through run_optimization's call
sequence without a GPU) via explicit injection ``BayesianOptimizer(..., engine=OracleEngine())``.  The product
never constructs this; its default engine is the HIP one, which raises when libgpx.so or the GPU is absent.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from bayesianoptimizer_amd._capi import NotPositiveDefiniteError
from oracle import gp_oracle as O

KINDS = {"rbf": O.RBF, "matern52": O.MATERN52, "scale_linear_matern52": O.SCALE_LINEAR_MATERN52}
ACQS = {"ei": O.ACQ_EI, "logei": O.ACQ_LOGEI, "ucb": O.ACQ_UCB, "variance": O.ACQ_VARIANCE}


def to_oracle_params(p, d):
    kind = KINDS[p.kind] if isinstance(p.kind, str) else int(p.kind)
    return O.KernelParams(kind, np.array(p.lengthscales(d)), outputscale=p.outputscale, noise=p.noise,
                          const_mean=p.const_mean, linear_variance=np.array(p.linear_variances(d)), jitter=p.jitter)


@dataclass
class OState:
    st: O.GPState
    alpha: torch.Tensor
    n: int
    nrhs: int
    params: object
    info: int = 0  # 0 or failing pivot + 1 (fit_outputs with check=False)


class OracleEngine:
    device = torch.device("cpu")

    def __init__(self):
        self.calls = {"fit": 0, "posterior": 0, "acquire": 0}

    def fit(self, X, Y, params, check=True, out=None, capacity=0, inverse=False):
        self.calls["fit"] += 1
        self.calls["fit_n"] = self.calls.get("fit_n", []) + [int(np.asarray(X).shape[0])]
        X = torch.as_tensor(X, dtype=torch.float64).cpu().numpy()
        Y = torch.as_tensor(Y, dtype=torch.float64).cpu().numpy()
        if Y.ndim == 1:
            Y = Y[:, None]
        try:
            st = O.fit(X, Y, to_oracle_params(params, X.shape[1]))
        except O.NotPDError as e:
            raise NotPositiveDefiniteError(e.pivot)
        return OState(st, torch.tensor(st.alpha.reshape(X.shape[0], -1)), X.shape[0], Y.shape[1], params)

    def fit_outputs(self, X, Y, params, check=True, out=None, inverse=False):
        """T independent outputs on one X, one parameter set each (GPEngine.fit_outputs)."""
        self.calls["fit_outputs"] = self.calls.get("fit_outputs", 0) + 1
        X = torch.as_tensor(X, dtype=torch.float64).cpu().numpy()
        Y = torch.as_tensor(Y, dtype=torch.float64).cpu().numpy()
        states = []
        for t, p in enumerate(params):
            try:
                st = O.fit(X, Y[:, t], to_oracle_params(p, X.shape[1]))
                states.append(OState(st, torch.tensor(st.alpha.reshape(-1, 1)), X.shape[0], 1, p))
            except O.NotPDError as e:
                if check:
                    raise NotPositiveDefiniteError(e.pivot)
                dummy = O.GPState(X=X, L=np.eye(X.shape[0]), alpha=np.zeros(X.shape[0]), params=None)
                states.append(OState(dummy, torch.zeros((X.shape[0], 1)), X.shape[0], 1, p, info=e.pivot + 1))
        return states

    @staticmethod
    def batch_info(states):
        return np.array([s.info for s in states], dtype=np.int64)

    def acquire_multi(self, states, Xs, kind="logei", best_f=0.0, beta=4.0, weights=None, y_mean=None, y_scale=None,
                      index_offset=0, return_scores=False):
        self.calls["acquire_multi"] = self.calls.get("acquire_multi", 0) + 1
        Xs = torch.as_tensor(Xs, dtype=torch.float64).cpu().numpy()
        T = len(states)
        w = np.ones(T) if weights is None else np.asarray(weights, dtype=np.float64)
        mu, var = O.objective_posterior([s.st for s in states], Xs, w, y_mean, y_scale)
        scores = O.acquisition(mu, var, ACQS[kind] if isinstance(kind, str) else int(kind), best_f, beta)
        v, i = O.argmax_lowest(scores)
        out = (torch.tensor([v], dtype=torch.float64), torch.tensor([i + index_offset], dtype=torch.int64))
        return out + (torch.tensor(scores),) if return_scores else out

    def mll_value_grad_outputs(self, X, Y, params, jitters=(0.0, 1e-8, 1e-7, 1e-6), states=None):
        self.calls["mll"] = self.calls.get("mll", 0) + 1
        Y = torch.as_tensor(Y, dtype=torch.float64)
        return [self.mll_value_grad(X, Y[:, t], p, jitters)[0] for t, p in enumerate(params)], None

    def mll_value_grad(self, X, Y, params, jitters=(0.0, 1e-8, 1e-7, 1e-6), state=None):
        self.calls["mll"] = self.calls.get("mll", 0) + 1
        self.calls["mll_n"] = self.calls.get("mll_n", set()) | {int(np.asarray(X).shape[0])}
        X = torch.as_tensor(X, dtype=torch.float64).cpu().numpy()
        Y = torch.as_tensor(Y, dtype=torch.float64).cpu().numpy()
        err = None
        for jit in jitters:
            try:
                return O.mll_value_grad(X, Y, to_oracle_params(params.replace(jitter=params.jitter + jit), X.shape[1])), None
            except O.NotPDError as e:
                err = NotPositiveDefiniteError(e.pivot)
        raise err

    def posterior(self, state, Xs, y_mean=None, y_scale=None):
        self.calls["posterior"] += 1
        Xs = torch.as_tensor(Xs, dtype=torch.float64).cpu().numpy()
        T = state.nrhs
        ym = np.zeros(T) if y_mean is None else np.asarray(y_mean, dtype=np.float64)
        ys = np.ones(T) if y_scale is None else np.asarray(y_scale, dtype=np.float64)
        mu, var = O.posterior(state.st, Xs)
        mu = mu.reshape(Xs.shape[0], T)
        var_std = var
        mean = ym + ys * mu
        var0 = np.maximum(var_std * ys[0] ** 2, O.BOTORCH_MIN_VAR)
        return torch.tensor(mean), torch.tensor(var0)

    def acquire(self, state, Xs, kind="logei", best_f=0.0, beta=4.0, y_mean=0.0, y_scale=1.0, alpha=None,
                index_offset=0, return_scores=False):
        self.calls["acquire"] += 1
        Xs = torch.as_tensor(Xs, dtype=torch.float64).cpu().numpy()
        a = state.alpha[:, 0] if alpha is None else torch.as_tensor(alpha)
        st1 = O.GPState(X=state.st.X, L=state.st.L, alpha=a.cpu().numpy()[: state.n], params=state.st.params)
        mu, var = O.posterior(st1, Xs, y_mean, y_scale)
        scores = O.acquisition(mu, var, ACQS[kind] if isinstance(kind, str) else int(kind), best_f, beta)
        v, i = O.argmax_lowest(scores)
        out = (torch.tensor([v], dtype=torch.float64), torch.tensor([i + index_offset], dtype=torch.int64))
        return out + (torch.tensor(scores),) if return_scores else out

    def moments_grad(self, state, Xs, q=1, alpha=None):
        self.calls["moments_grad"] = self.calls.get("moments_grad", 0) + 1
        Xs = torch.as_tensor(Xs, dtype=torch.float64).cpu().numpy()
        a = state.alpha[:, 0] if alpha is None else torch.as_tensor(alpha)
        out = O.moments_grad(state.st, Xs, q, a.cpu().numpy()[: state.n])
        return tuple(torch.tensor(v) for v in out)

    def argmax_combine(self, vals, idx):
        v, i = O.combine_argmax(list(zip(vals.tolist(), idx.tolist())))
        return torch.tensor([v]), torch.tensor([i])

    def topk(self, scores, k):
        self.calls["topk"] = self.calls.get("topk", 0) + 1
        v, i = O.topk_desc(torch.as_tensor(scores).cpu().numpy(), int(k))
        return torch.tensor(v), torch.tensor(i)

    def fps(self, X, k, start):
        self.calls["fps"] = self.calls.get("fps", 0) + 1
        return torch.tensor(O.farthest_point_sampling(torch.as_tensor(X).cpu().numpy(), int(k), int(start)))

    def append(self, state, X, Y, check=True):
        self.calls["append"] = self.calls.get("append", 0) + 1
        X = torch.as_tensor(X, dtype=torch.float64).cpu().numpy()
        Y = torch.as_tensor(Y, dtype=torch.float64).cpu().numpy()
        if Y.ndim == 1:
            Y = Y[:, None]
        try:
            st = O.append(state.st, X, Y)
        except O.NotPDError as e:
            raise NotPositiveDefiniteError(e.pivot)
        return OState(st, torch.tensor(st.alpha.reshape(X.shape[0], -1)), X.shape[0], Y.shape[1], state.params)
