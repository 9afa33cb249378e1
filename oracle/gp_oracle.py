"""CPU oracle for the exact-GP posterior hot path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it.  The shipped path (``bayesianoptimizer_amd``)
never imports anything under ``oracle/`` and fails loudly when its HIP library is missing.

What it restates (fp64, NumPy/SciPy):

* a3  Gram build ``K(X,X) + (noise + jitter) I`` for the three kernels the reference uses:
      RBF (BoTorch >= 0.12 ``SingleTaskGP`` default covariance, reached from
      ``optimization/Bayesian.py:91`` and ``optimization/Bayesian1.py:109``), Matérn-5/2, and
      ``ScaleKernel(LinearKernel + MaternKernel(nu=2.5))`` (``optimization/Bayesian6.py:471-473``,
      ``optimization/Bayesian7.py:162-166``).  [upstream] GPyTorch kernel formulas.
* a4  Cholesky ``K = L L^T`` with NOT_PD reporting of the failing pivot (the reference retries
      with a larger jitter, ``optimization/Bayesian6.py:481-488``).
* a5  ``alpha = K^{-1} (y - m)``, m = ConstantMean.
* a6  Posterior ``mu = m + k*^T alpha``, ``var = k** - ||L^{-1} k*||^2`` with GPyTorch's
      double-precision variance floor (1e-10) and BoTorch's ``min_var`` floor (1e-12), as used by
      ``model.posterior(X).mean/.variance`` (``optimization/Bayesian2.py:169-171``,
      ``optimization/Bayesian6.py:615-617``).
* a7  Analytic EI / LogEI / UCB / posterior-variance scores (BoTorch analytic acquisition
      formulas [upstream]; the reference's qLogEI call site is ``optimization/Bayesian.py:100-101``,
      the variance-sum pool scan is ``optimization/Bayesian7.py:664-671``).
* a8  Argmax with the lowest index winning ties (``optimization/Bayesian.py:117``,
      ``optimization/Bayesian7.py:681,724-727``).
* §8f row 3: the bordered-Cholesky append of new observations (``append``), equal to a refit.
* §8f row 4: q-batch posterior moments and their candidate gradients (``moments_grad``) and the MC qLogEI of
      the optimize_acqf refinement (``qlogei``), optimization/Bayesian.py:96-113.
* §8f row 1: -log p(y) and its gradient w.r.t. the kernel hyperparameters (``mll_value_grad``).
* a9 / §8f row 2: the batched SVGP predictive of ``optimization/Bayesian7.py:543-563,664-671`` (gpytorch's whitened
      ``VariationalStrategy`` [upstream]: mean = c + k*^T L^{-T} m, var = k** + k*^T L^{-T}(S S^T - I)L^{-1} k* +
      noise), the torch.topk of ``:681`` (stable, descending) and ``farthest_point_sampling`` of ``:82-106``
      (``svgp_predict``, ``topk_desc``, ``farthest_point_sampling``).
* a1/a2 input/output transforms of ``optimization/Bayesian7.py:181-190,363-385``.

Parity status: **parity unpinned**.  The reference delegates this arithmetic to GPyTorch /
BoTorch / linear_operator, which are not installed here and not vendored under the reference,
and the reference holds no tests or golden vectors for this path.  The
oracle is therefore pinned by closed-form known-answer tests (tests/test_oracle.py) and by the
golden fixtures it generates itself (tests/golden/make_golden.py); parity is defined against the
exact-Cholesky formulation (no CG/Lanczos/LOVE, no MC sampling), see DESIGN.md §3.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np
import scipy.linalg as sla
from scipy.special import erfcx, ndtr

RBF = 0
MATERN52 = 1
SCALE_LINEAR_MATERN52 = 2

ACQ_EI = 0
ACQ_LOGEI = 1
ACQ_UCB = 2
ACQ_VARIANCE = 3

# GPyTorch settings.min_variance for float64 [upstream]; BoTorch analytic min_var [upstream].
GPYTORCH_MIN_VAR_F64 = 1e-10
BOTORCH_MIN_VAR = 1e-12


@dataclass
class KernelParams:
    """Fixed GP hyperparameters (mirrors bayesianoptimizer_amd.KernelParams)."""

    kind: int
    lengthscale: np.ndarray
    outputscale: float = 1.0
    noise: float = 1e-4
    const_mean: float = 0.0
    linear_variance: Optional[np.ndarray] = None
    jitter: float = 0.0
    cov_fp32: bool = False  # BASELINE configs[4]: covariance evaluated in fp32, widened before factorisation
    # "difference": sum_k ((a_k - b_k)/l_k)^2, the form the GPU kernels compute; "expanded": GPyTorch's
    # ||a||^2 + ||b||^2 - 2 a.b on inputs centred by mean(X1), clamped >= 0, diagonal zeroed for K(X, X) [upstream]
    # (used only to bound the formulation gap to GPyTorch, tests/test_oracle.py)
    dist_form: str = "difference"

    def __post_init__(self):
        self.lengthscale = np.asarray(self.lengthscale, dtype=np.float64).reshape(-1)
        if self.linear_variance is None:
            self.linear_variance = np.ones_like(self.lengthscale)
        self.linear_variance = np.asarray(self.linear_variance, dtype=np.float64).reshape(-1)
        if self.linear_variance.size == 1 and self.lengthscale.size > 1:
            self.linear_variance = np.full_like(self.lengthscale, self.linear_variance[0])


def botorch_default_lengthscale(d: int) -> float:
    """Mode of BoTorch's dimension-scaled LogNormal(sqrt2 + 0.5 log d, sqrt3) prior [upstream]."""
    return math.exp(math.sqrt(2.0) + 0.5 * math.log(d) - 3.0)


# ---------------------------------------------------------------------------------------------
# a3: kernels
# ---------------------------------------------------------------------------------------------
def _sqdist_scaled(X1: np.ndarray, X2: np.ndarray, ls: np.ndarray) -> np.ndarray:
    """Squared distances of lengthscale-scaled inputs, difference form sum_k ((a_k-b_k)/l_k)^2.

    The GPU Gram/K* kernels accumulate the same per-dimension terms in the same order (k = 0..d-1),
    so the two agree to rounding of the final exp.  [upstream] GPyTorch uses the expanded form
    ||a||^2+||b||^2-2a.b on mean-centred inputs; that differs by O(eps) and is documented in
    DESIGN.md as part of the parity definition.
    """
    A = X1 / ls
    B = X2 / ls
    out = np.zeros((A.shape[0], B.shape[0]), dtype=np.float64)
    for k in range(A.shape[1]):
        diff = A[:, k:k + 1] - B[None, :, k]
        out += diff * diff
    return out


def _sqdist_scaled_expanded(X1: np.ndarray, X2: np.ndarray, ls: np.ndarray, same: bool) -> np.ndarray:
    """GPyTorch's Distance._sq_dist [upstream] restated: scale by the lengthscales, centre both inputs by mean(X1),
    r2 = ||a||^2 + ||b||^2 - 2 a.b, clamped at 0, the diagonal set to 0 when X1 is X2."""
    A = X1 / ls
    B = X2 / ls
    adj = A.mean(axis=0, keepdims=True)
    A = A - adj
    B = B - adj
    r2 = (A * A).sum(1)[:, None] + (B * B).sum(1)[None, :] - 2.0 * (A @ B.T)
    if same:
        np.fill_diagonal(r2, 0.0)
    return np.maximum(r2, 0.0)


def kernel_matrix(X1: np.ndarray, X2: np.ndarray, p: KernelParams) -> np.ndarray:
    """k(X1, X2) without noise.  Formulas per GPyTorch RBFKernel/MaternKernel/LinearKernel/ScaleKernel."""
    same = X1 is X2
    X1 = np.asarray(X1, dtype=np.float64)
    X2 = np.asarray(X2, dtype=np.float64)
    if p.cov_fp32:
        return _kernel_matrix_f32(X1, X2, p)
    if p.dist_form == "expanded":
        r2 = _sqdist_scaled_expanded(X1, X2, p.lengthscale, same)
    else:
        r2 = _sqdist_scaled(X1, X2, p.lengthscale)
    if p.kind == RBF:
        return p.outputscale * np.exp(-0.5 * r2)
    r = np.sqrt(r2)
    s5r = math.sqrt(5.0) * r
    matern = (1.0 + s5r + (5.0 / 3.0) * r2) * np.exp(-s5r)
    if p.kind == MATERN52:
        return p.outputscale * matern
    if p.kind == SCALE_LINEAR_MATERN52:
        lin = (X1 * p.linear_variance) @ X2.T
        return p.outputscale * (lin + matern)
    raise ValueError(f"unknown kernel kind {p.kind}")


def _kernel_matrix_f32(X1, X2, p: KernelParams) -> np.ndarray:
    """fp32 evaluation: scaled inputs rounded to fp32, squared distance summed in fp32 (k = 0..d-1), exp and the
    Matern polynomial in fp32, widened to fp64 before the outputscale and the (fp64) linear part."""
    A = (X1 / p.lengthscale).astype(np.float32)
    B = (X2 / p.lengthscale).astype(np.float32)
    r2 = np.zeros((A.shape[0], B.shape[0]), dtype=np.float32)
    for k in range(A.shape[1]):
        diff = A[:, k:k + 1] - B[None, :, k]
        r2 += diff * diff
    if p.kind == RBF:
        return p.outputscale * np.exp(np.float32(-0.5) * r2).astype(np.float64)
    r = np.sqrt(r2)
    s5r = np.float32(math.sqrt(5.0)) * r
    m = ((np.float32(1.0) + s5r + np.float32(5.0 / 3.0) * r2) * np.exp(-s5r)).astype(np.float64)
    if p.kind == MATERN52:
        return p.outputscale * m
    lin = (X1 * p.linear_variance) @ X2.T
    return p.outputscale * (lin + m)


def kernel_diag(X: np.ndarray, p: KernelParams) -> np.ndarray:
    """k(x, x) for each row."""
    X = np.asarray(X, dtype=np.float64)
    if p.kind in (RBF, MATERN52):
        return np.full(X.shape[0], p.outputscale)
    lin = (X * X * p.linear_variance).sum(axis=1)
    return p.outputscale * (lin + 1.0)


def gram(X: np.ndarray, p: KernelParams) -> np.ndarray:
    """K(X,X) + (noise + jitter) I  (SURVEY §8a row a3)."""
    K = kernel_matrix(X, X, p)
    K[np.diag_indices_from(K)] += p.noise + p.jitter
    return K


# ---------------------------------------------------------------------------------------------
# a4/a5: factorisation and alpha
# ---------------------------------------------------------------------------------------------
class NotPDError(np.linalg.LinAlgError):
    def __init__(self, pivot: int):
        super().__init__(f"matrix not positive definite at pivot {pivot}")
        self.pivot = pivot


def cholesky(K: np.ndarray) -> np.ndarray:
    """Lower Cholesky factor; raises NotPDError(pivot) like the C-ABI's info = pivot + 1."""
    try:
        return sla.cholesky(K, lower=True, check_finite=False)
    except np.linalg.LinAlgError as e:  # scipy: "%d-th leading minor not positive definite"
        msg = str(e)
        piv = -1
        for tok in msg.split():
            if tok.rstrip("-th").isdigit():
                piv = int(tok.rstrip("-th")) - 1
                break
        raise NotPDError(piv) from e


@dataclass
class GPState:
    X: np.ndarray
    L: np.ndarray
    alpha: np.ndarray  # (n,) or (n, T)
    params: KernelParams


def fit(X: np.ndarray, y: np.ndarray, p: KernelParams) -> GPState:
    """One posterior update: Gram + Cholesky + alpha."""
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    K = gram(X, p)
    L = cholesky(K)
    alpha = sla.cho_solve((L, True), y - p.const_mean, check_finite=False)
    return GPState(X=X, L=L, alpha=alpha, params=p)


def psd_safe_jitters(jitter_val: float = 1e-4, retry: float = 1e-2, max_tries: int = 3):
    """Jitters the reference's exact fit tries in order (optimization/Bayesian6.py:482-488): GPyTorch's
    psd_safe_cholesky [upstream] factors without jitter, then with cholesky_jitter * 10^i, i < cholesky_max_tries = 3,
    under cholesky_jitter(jitter_val = 1e-4) (Bayesian6.py:66,483) and on failure under cholesky_jitter(1e-2) (:487)."""
    seq = [0.0]
    for base in (jitter_val, retry):
        for i in range(max_tries):
            j = base * 10.0 ** i
            if all(abs(j - s) > 1e-12 * j for s in seq):
                seq.append(j)
    return seq


def fit_with_jitter(X: np.ndarray, y: np.ndarray, p: KernelParams, jitters=None):
    """fit() with the first jitter of ``jitters`` (default psd_safe_jitters()) whose factorisation succeeds; returns
    (state, jitter, failed pivots of the earlier attempts).  Raises the last NotPDError when none succeeds."""
    failed = []
    last = None
    for jit in (psd_safe_jitters() if jitters is None else jitters):
        q = KernelParams(**{**p.__dict__, "jitter": jit})
        try:
            return fit(X, y, q), jit, failed
        except NotPDError as e:
            failed.append(e.pivot)
            last = e
    raise last


def append(state: GPState, X_all: np.ndarray, y_all: np.ndarray) -> GPState:
    """Incremental posterior update: the rows of X_all past ``state.X`` appended by a bordered
    Cholesky (L21 = K21 L11^{-T}, L22 = chol(K22 - L21 L21^T)) instead of the refit the reference runs every round
    after appending observations (optimization/Bayesian7.py:628-631,639; optimization/Bayesian.py:163-174).  Equal
    to ``fit(X_all, y_all, state.params)`` up to rounding; alpha is recomputed from all of y_all."""
    p = state.params
    X_all = np.asarray(X_all, dtype=np.float64)
    y_all = np.asarray(y_all, dtype=np.float64)
    n0 = state.X.shape[0]
    Xn = X_all[n0:]
    K21 = kernel_matrix(Xn, X_all[:n0], p)
    K22 = gram(Xn, p)
    L21 = sla.solve_triangular(state.L, K21.T, lower=True, check_finite=False).T
    try:
        L22 = cholesky(K22 - L21 @ L21.T)
    except NotPDError as e:
        raise NotPDError(n0 + e.pivot) from e
    n = X_all.shape[0]
    L = np.zeros((n, n))
    L[:n0, :n0] = state.L
    L[n0:, :n0] = L21
    L[n0:, n0:] = L22
    alpha = sla.cho_solve((L, True), y_all - p.const_mean, check_finite=False)
    return GPState(X=X_all, L=L, alpha=alpha, params=p)


# ---------------------------------------------------------------------------------------------
# §8f row 1: negative log marginal likelihood and its hyperparameter gradient
# ---------------------------------------------------------------------------------------------
def kernel_grads(X: np.ndarray, p: KernelParams) -> dict:
    """dK/d theta (n x n each, noise excluded) for the natural hyperparameters of ``p`` (fp64).

    RBF  k = s exp(-r^2/2):                 dk/dl_k = k q_k / l_k,  dk/ds = exp(-r^2/2)
    M52  k = s (1+sqrt5 r+5r^2/3) e^{-sqrt5 r}: dk/dl_k = s (5/3)(1+sqrt5 r) e^{-sqrt5 r} q_k / l_k,
                                               dk/ds = (1+sqrt5 r+5r^2/3) e^{-sqrt5 r}
    +lin k = s (sum_k v_k x_k x'_k + M52):   dk/dv_k = s x_k x'_k,  dk/ds += sum_k v_k x_k x'_k
    with q_k = ((x_k - x'_k) / l_k)^2 (GPyTorch RBFKernel / MaternKernel / LinearKernel / ScaleKernel [upstream]).
    """
    X = np.asarray(X, dtype=np.float64)
    ls = p.lengthscale
    q = [((X[:, k:k + 1] - X[None, :, k]) / ls[k]) ** 2 for k in range(X.shape[1])]
    r2 = np.zeros_like(q[0])
    for qk in q:
        r2 += qk
    if p.kind == RBF:
        base = np.exp(-0.5 * r2)
        kfac = p.outputscale * base
    else:
        r = np.sqrt(r2)
        ex = np.exp(-math.sqrt(5.0) * r)
        base = (1.0 + math.sqrt(5.0) * r + (5.0 / 3.0) * r2) * ex
        kfac = p.outputscale * (5.0 / 3.0) * (1.0 + math.sqrt(5.0) * r) * ex
    out = {"lengthscale": [kfac * q[k] / ls[k] for k in range(X.shape[1])]}
    if p.kind == SCALE_LINEAR_MATERN52:
        out["linear_variance"] = [p.outputscale * np.outer(X[:, k], X[:, k]) for k in range(X.shape[1])]
        base = base + (X * p.linear_variance) @ X.T
    out["outputscale"] = base
    return out


def mll_value_grad(X: np.ndarray, y: np.ndarray, p: KernelParams) -> dict:
    """-log p(Y) = sum_t [1/2 (y_t-m)^T alpha_t] + T (sum log L_ii + n/2 log 2pi) and its gradient
    1/2 sum_ij (T K^{-1} - sum_t alpha_t alpha_t^T)_ij dK_ij/d theta, d/dm = -sum alpha, for T outputs sharing
    the covariance (T = 1: the quantity ExactMarginalLogLikelihood differentiates inside fit_gpytorch_mll
    [upstream], reached from optimization/Bayesian.py:92-93, optimization/Bayesian6.py:480-488), before the
    1/n scaling and priors."""
    X = np.asarray(X, dtype=np.float64)
    Y = np.asarray(y, dtype=np.float64)
    Y = Y.reshape(-1, 1) if Y.ndim == 1 else Y
    n, T = Y.shape
    st = fit(X, Y, p)
    L, alpha = st.L, st.alpha
    quad = 0.5 * float(((Y - p.const_mean) * alpha).sum())
    logdet = 2.0 * float(np.log(np.diag(L)).sum())
    Kinv = sla.cho_solve((L, True), np.eye(n), check_finite=False)
    G = 0.5 * (T * Kinv - alpha @ alpha.T)
    dk = kernel_grads(X, p)
    d = X.shape[1]
    res = {
        "nll": quad + T * (0.5 * logdet + 0.5 * n * math.log(2.0 * math.pi)),
        "quad": quad,
        "logdet": logdet,
        "noise": float(np.trace(G)),
        "outputscale": float((G * dk["outputscale"]).sum()),
        "const_mean": -float(alpha.sum()),
        "lengthscale": np.array([(G * dk["lengthscale"][k]).sum() for k in range(d)]),
        "linear_variance": (np.array([(G * dk["linear_variance"][k]).sum() for k in range(d)])
                            if p.kind == SCALE_LINEAR_MATERN52 else np.zeros(d)),
    }
    return res


# ---------------------------------------------------------------------------------------------
# a6: posterior
# ---------------------------------------------------------------------------------------------
def posterior(state: GPState, Xs: np.ndarray, y_mean: float = 0.0, y_scale: float = 1.0):
    """Posterior mean/variance at Xs, untransformed by (y_mean, y_scale) like Standardize.

    Variance floor order: GPyTorch clamps the standardized predictive variance at 1e-10 (double),
    Standardize.untransform multiplies by y_scale^2, then BoTorch clamps at 1e-12 [upstream].
    """
    p = state.params
    Ks = kernel_matrix(state.X, Xs, p)  # (n, m)
    mu = p.const_mean + Ks.T @ state.alpha
    V = sla.solve_triangular(state.L, Ks, lower=True, check_finite=False)
    var = kernel_diag(Xs, p) - np.einsum("ij,ij->j", V, V)
    var = np.maximum(var, GPYTORCH_MIN_VAR_F64)
    mu = y_mean + y_scale * mu
    var = np.maximum(var * (y_scale * y_scale), BOTORCH_MIN_VAR)
    return mu, var


def fit_outputs(X: np.ndarray, Y: np.ndarray, params: Sequence[KernelParams]):
    """T independent GPs on one X (Y: n x T, one KernelParams per output): the reference's multi-output SingleTaskGP,
    optimization/Bayesian1.py:108-116 (a batch of independent GPs, each with its own hyperparameters [upstream])."""
    Y = np.asarray(Y, dtype=np.float64)
    return [fit(X, Y[:, t], params[t]) for t in range(Y.shape[1])]


def objective_posterior(states: Sequence[GPState], Xs: np.ndarray, weights, y_mean=None, y_scale=None):
    """Posterior of f = sum_t w_t (y_mean_t + y_scale_t g_t) over independent outputs g_t: mean sum_t w_t (y_mean_t +
    y_scale_t mu_t), variance sum_t w_t^2 y_scale_t^2 var_t (GPyTorch's 1e-10 floor per output, BoTorch's 1e-12 on the
    sum [upstream]) — BoTorch's ScalarizedPosteriorTransform of a batched multi-output posterior, analytic form."""
    T = len(states)
    ym = np.zeros(T) if y_mean is None else np.asarray(y_mean, dtype=np.float64)
    ys = np.ones(T) if y_scale is None else np.asarray(y_scale, dtype=np.float64)
    w = np.asarray(weights, dtype=np.float64)
    mu = np.zeros(Xs.shape[0])
    var = np.zeros(Xs.shape[0])
    for t, st in enumerate(states):
        p = st.params
        Ks = kernel_matrix(st.X, Xs, p)
        m_t = (p.const_mean + Ks.T @ st.alpha).reshape(-1)  # alpha: (n,) or one column (n, 1)
        V = sla.solve_triangular(st.L, Ks, lower=True, check_finite=False)
        v_t = np.maximum(kernel_diag(Xs, p) - np.einsum("ij,ij->j", V, V), GPYTORCH_MIN_VAR_F64)
        mu += w[t] * (ym[t] + ys[t] * m_t)
        var += w[t] * w[t] * (ys[t] * ys[t] * v_t)
    return mu, np.maximum(var, BOTORCH_MIN_VAR)


# ---------------------------------------------------------------------------------------------
# a7: analytic acquisition (BoTorch analytic forms, restated)
# ---------------------------------------------------------------------------------------------
_LOG_SQRT_2PI = 0.5 * math.log(2.0 * math.pi)
_LOG_SQRT_PI_DIV_2 = 0.5 * math.log(math.pi / 2.0)
_INV_SQRT_2 = 1.0 / math.sqrt(2.0)
_NEG_INV_SQRT_EPS_F64 = -1.0 / math.sqrt(np.finfo(np.float64).eps)


def _phi(u):
    return np.exp(-0.5 * u * u) / math.sqrt(2.0 * math.pi)


def _Phi(u):
    return ndtr(u)


def _log1mexp(x):
    """log(1 - exp(x)) for x < 0 (Maechler's two-branch form)."""
    x = np.asarray(x, dtype=np.float64)
    return np.where(x > -math.log(2.0), np.log(-np.expm1(np.minimum(x, -1e-300))),
                    np.log1p(-np.exp(np.minimum(x, 0.0))))


def ei_helper(u):
    return _phi(u) + u * _Phi(u)


def log_ei_helper(u):
    """log(phi(u) + u Phi(u)), stable for very negative u (two-branch form, bound = -1)."""
    u = np.asarray(u, dtype=np.float64)
    upper = np.log(ei_helper(np.maximum(u, -1.0)))
    u_lo = np.minimum(u, -1.0)
    u_eps = np.maximum(u_lo, _NEG_INV_SQRT_EPS_F64)
    w = np.log(erfcx(-u_eps * _INV_SQRT_2) * np.abs(u_eps)) + _LOG_SQRT_PI_DIV_2
    log_phi = -0.5 * u * u - _LOG_SQRT_2PI
    lower = log_phi + np.where(u > _NEG_INV_SQRT_EPS_F64, _log1mexp(w), -2.0 * np.log(np.abs(u_lo)))
    return np.where(u > -1.0, upper, lower)


def acquisition(mu, var, kind: int, best_f: float = 0.0, beta: float = 4.0):
    """Score per candidate; higher is better (maximisation)."""
    mu = np.asarray(mu, dtype=np.float64)
    var = np.asarray(var, dtype=np.float64)
    sigma = np.sqrt(var)
    if kind == ACQ_EI:
        u = (mu - best_f) / sigma
        return sigma * ei_helper(u)
    if kind == ACQ_LOGEI:
        u = (mu - best_f) / sigma
        return log_ei_helper(u) + np.log(sigma)
    if kind == ACQ_UCB:
        return mu + math.sqrt(beta) * sigma
    if kind == ACQ_VARIANCE:
        return var
    raise ValueError(f"unknown acquisition {kind}")


# ---------------------------------------------------------------------------------------------
# §8f row 4: q-batch posterior moments, their candidate gradients, MC qLogEI (optimize_acqf refinement,
# optimization/Bayesian.py:96-113, optimization/Bayesian2.py:218-245; BoTorch/GPyTorch autograd [upstream])
# ---------------------------------------------------------------------------------------------
def kernel_grad_first(Xa: np.ndarray, Xb: np.ndarray, p: KernelParams) -> np.ndarray:
    """d k(a, b) / d a_j for every pair: (na, nb, d)."""
    ls = np.asarray(p.lengthscale, dtype=np.float64)
    diff = (Xa[:, None, :] / ls - Xb[None, :, :] / ls) / ls  # (a_j - b_j) / l_j^2
    r2 = _sqdist_scaled(Xa, Xb, ls)
    if p.kind == RBF:
        coef = -p.outputscale * np.exp(-0.5 * r2)
    else:
        r = np.sqrt(r2)
        coef = -p.outputscale * (5.0 / 3.0) * (1.0 + math.sqrt(5.0) * r) * np.exp(-math.sqrt(5.0) * r)
    g = coef[:, :, None] * diff
    if p.kind == SCALE_LINEAR_MATERN52:
        g = g + p.outputscale * (np.asarray(p.linear_variance)[None, None, :] * Xb[None, :, :])
    return g


def moments_grad(state: GPState, Xs: np.ndarray, q: int, alpha: Optional[np.ndarray] = None):
    """NumPy restatement of gpx_moments_grad_f64: mean (m), dmean (m, d), cov (m, q), dcov (m, d, q)."""
    p = state.params
    alpha = state.alpha if alpha is None else alpha
    alpha = alpha[:, 0] if alpha.ndim == 2 else alpha
    m, d = Xs.shape
    Ks = kernel_matrix(state.X, Xs, p)  # (n, m)
    S = sla.cho_solve((state.L, True), Ks, check_finite=False)  # K^{-1} K*
    G = kernel_grad_first(Xs, state.X, p)  # (m, n, d)
    mean = p.const_mean + Ks.T @ alpha
    dmean = np.einsum("anj,n->aj", G, alpha)
    cov = np.empty((m, q))
    dcov = np.empty((m, d, q))
    for a in range(m):
        b0 = (a // q) * q
        cols = slice(b0, b0 + q)
        kp = kernel_matrix(Xs[a:a + 1], Xs[cols], p)[0]
        gp = kernel_grad_first(Xs[a:a + 1], Xs[cols], p)[0]  # (q, d)
        cov[a] = kp - Ks[:, a] @ S[:, cols]
        dcov[a] = gp.T - G[a].T @ S[:, cols]
    return mean, dmean, cov, dcov


def sobol_normal_base_samples(S: int, q: int, seed: int) -> np.ndarray:
    """The base samples of the product's SobolQMCNormalSampler (torch SobolEngine, scramble, seed; inverse cdf)."""
    import torch
    u = torch.quasirandom.SobolEngine(dimension=q, scramble=True, seed=seed).draw(S, dtype=torch.float64).numpy()
    eps = np.finfo(np.float64).eps
    v = 0.5 + (1.0 - eps) * (u - 0.5)
    from scipy.special import erfinv
    return erfinv(2.0 * v - 1.0) * math.sqrt(2.0)


def qlogei(mu: np.ndarray, Sigma: np.ndarray, z: np.ndarray, best_f: float, fat: bool = True,
           tau_max: float = 1e-2, tau_relu: float = 1e-6) -> np.ndarray:
    """MC qLogEI of q-batches: mu (B, q), Sigma (B, q, q), base samples z (S, q) -> (B,)."""
    from scipy.special import logsumexp
    L = np.linalg.cholesky(0.5 * (Sigma + np.swapaxes(Sigma, 1, 2)))
    f = mu[None] + np.einsum("bij,sj->sbi", L, z)
    y = (f - best_f) / tau_relu
    if fat:
        sp = np.logaddexp(0.0, y)
        li = math.log(tau_relu) + np.log(sp + 0.1 / (1.0 + y * y))
    else:
        li = math.log(tau_relu) + np.where(y > -37.0, np.log(np.logaddexp(0.0, np.maximum(y, -37.0))), y)
    qred = tau_max * logsumexp(li / tau_max, axis=-1)
    return logsumexp(qred, axis=0) - math.log(z.shape[0])


# ---------------------------------------------------------------------------------------------
# a8: argmax (lowest index wins ties; NaN never wins)
# ---------------------------------------------------------------------------------------------
def argmax_lowest(scores: np.ndarray):
    s = np.asarray(scores, dtype=np.float64)
    s = np.where(np.isnan(s), -np.inf, s)
    idx = int(np.argmax(s))  # numpy returns the first occurrence of the max
    return float(s[idx]), idx


def acquire_argmax(state: GPState, Xs: np.ndarray, kind: int, best_f: float = 0.0,
                   beta: float = 4.0, y_mean: float = 0.0, y_scale: float = 1.0,
                   chunk: int = 8192):
    """Candidate sweep + argmax.  Returns (best_value, best_index, scores)."""
    scores = np.empty(Xs.shape[0], dtype=np.float64)
    for s in range(0, Xs.shape[0], chunk):
        mu, var = posterior(state, Xs[s:s + chunk], y_mean, y_scale)
        scores[s:s + chunk] = acquisition(mu, var, kind, best_f, beta)
    v, i = argmax_lowest(scores)
    return v, i, scores


def combine_argmax(records: Sequence[tuple]):
    """Deterministic reduction of (value, global_index) records: max value, then lowest index."""
    best = (-np.inf, np.iinfo(np.int64).max)
    for v, i in records:
        v = -np.inf if np.isnan(v) else v
        if v > best[0] or (v == best[0] and i < best[1]):
            best = (v, i)
    return best


# ---------------------------------------------------------------------------------------------
# a1/a2: transforms (optimization/Bayesian7.py:181-190, 363-385)
# ---------------------------------------------------------------------------------------------
def log_standardize_inputs(X_unit, bounds, mean=None, std=None, std_floor=1e-6):
    b = np.asarray(bounds, dtype=np.float64)
    lo, hi = b[:, 0], b[:, 1]
    X_phys = X_unit * (hi - lo) + lo
    X_log = np.log(np.maximum(X_phys, 1e-6))
    if mean is None:
        mean = X_log.mean(axis=0, keepdims=True)
        std = np.maximum(X_log.std(axis=0, ddof=1, keepdims=True), std_floor)
    return (X_log - mean) / std, mean, std


def standardize(Y):
    """BoTorch Standardize: (y - mean) / std with unbiased std [upstream]."""
    Y = np.asarray(Y, dtype=np.float64)
    m = Y.mean(axis=0)
    s = Y.std(axis=0, ddof=1)
    s = np.where(s >= 1e-8, s, 1.0)
    return (Y - m) / s, m, s


# ---------------------------------------------------------------------------------------------
# synthetic workload of SURVEY §8d
# ---------------------------------------------------------------------------------------------
def synthetic_problem(n: int, d: int, seed: int, noise_sd: float = 0.01):
    rng = np.random.default_rng(seed)
    X = rng.random((n, d))
    y = np.sin(6.0 * X).sum(axis=1) + noise_sd * rng.standard_normal(n)
    sd = y.std()
    y = (y - y.mean()) / (sd if sd > 0 else 1.0)
    return X, y


def sobol_candidates(m: int, d: int, seed: int):
    from scipy.stats import qmc
    eng = qmc.Sobol(d, scramble=True, seed=seed)
    k = int(math.ceil(math.log2(max(m, 1))))
    return eng.random_base2(k)[:m]


# ---------------------------------------------------------------------------------------------
# a9 / §8f row 2: batched SVGP predictive + pool-scan selection (optimization/Bayesian7.py)
# ---------------------------------------------------------------------------------------------
VARIATIONAL_JITTER_F32 = 1e-4  # gpytorch settings.variational_cholesky_jitter, float32 [upstream]


def svgp_predict(Z, vmean, vchol, params: Sequence[KernelParams], Xs, jitter=VARIATIONAL_JITTER_F32,
                 min_var=GPYTORCH_MIN_VAR_F64):
    """Per task t (``optimization/Bayesian7.py:137-178`` BatchSVGP, whitened VariationalStrategy [upstream]):
    L = chol(K_ZZ + jitter I), A = L^{-1} K_ZX, mean = c_t + A^T m_t,
    var = k(x, x) + colsum(A * ((S S^T - I) A)) + noise_t  (S = tril(chol_variational_covar)),
    floored at ``min_var`` (gpytorch MultivariateNormal.variance [upstream]).  Returns mean, var (m x T) and the
    pool-scan score sum_t var (``optimization/Bayesian7.py:671``)."""
    T = len(params)
    Xs = np.asarray(Xs, dtype=np.float64)
    mean = np.empty((Xs.shape[0], T))
    var = np.empty((Xs.shape[0], T))
    for t in range(T):
        p = params[t]
        Zt = np.asarray(Z[t], dtype=np.float64)
        Kzz = kernel_matrix(Zt, Zt, p)
        Kzz[np.diag_indices_from(Kzz)] += jitter
        L = cholesky(Kzz)
        A = sla.solve_triangular(L, kernel_matrix(Zt, Xs, p), lower=True, check_finite=False)
        S = np.tril(np.asarray(vchol[t], dtype=np.float64))
        SA = S.T @ A
        mean[:, t] = p.const_mean + A.T @ np.asarray(vmean[t], dtype=np.float64)
        v = kernel_diag(Xs, p) - np.einsum("ij,ij->j", A, A) + np.einsum("ij,ij->j", SA, SA) + p.noise
        var[:, t] = np.maximum(v, min_var)
    return mean, var, var.sum(axis=1)


def topk_desc(scores, k):
    """The k largest scores, descending; equal scores keep the lower index first; NaN ranks last (torch.topk of
    ``optimization/Bayesian7.py:681`` with a deterministic tie order)."""
    s = np.asarray(scores, dtype=np.float64)
    key = np.where(np.isnan(s), -np.inf, s)
    order = np.argsort(-key, kind="stable")[:k]
    return key[order], order


def farthest_point_sampling(X, k, start):
    """Greedy FPS (``optimization/Bayesian7.py:82-106``) from index ``start``: squared Euclidean distances (fp64,
    summed over dimensions in order), argmax with the lowest index among ties (torch.argmax).  Returns the selected
    indices in selection order."""
    X = np.asarray(X, dtype=np.float64)

    def sqdist(c):
        d2 = np.zeros(X.shape[0])
        for j in range(X.shape[1]):  # dimension order, like the device loop
            d2 += (X[:, j] - X[c, j]) ** 2
        return d2

    idx = [int(start)]
    dist = sqdist(start)
    for _ in range(1, k):
        far = int(np.argmax(dist))
        idx.append(far)
        dist = np.minimum(dist, sqdist(far))
    return np.asarray(idx, dtype=np.int64)
