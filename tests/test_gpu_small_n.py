"""Fused small-n sweep (sweep_small_kernel: npad <= 256, d <= 16, 1..8 outputs, fp64 covariance build; n = 257..384
cases check the boundary, where both sides take the K* + trmm path): every case is checked against the oracle at the parity tolerances of tests/test_gpu_parity.py, and against the unfused K* + trmm path
of the same library (handle option sweep_fused = 0, GPX_OPT_SWEEP_FUSED) — the two paths sum in different orders, so they agree to the
same 1e-9 tolerance, and their argmax agrees exactly or at a reported tie."""
import numpy as np
import pytest

from oracle import gp_oracle as O
from tests.test_gpu_parity import check_argmax, check_posterior, pair, t

pytestmark = pytest.mark.gpu
ACQS = {"ei": O.ACQ_EI, "logei": O.ACQ_LOGEI, "ucb": O.ACQ_UCB, "variance": O.ACQ_VARIANCE}


def _run(engine, st, Xs, acq, best_f, fused):
    engine.set_option("sweep_fused", 1 if fused else 0)
    try:
        mu, var = engine.posterior(st, t(Xs))
        bv, bi, sg = engine.acquire(st, t(Xs), acq, best_f=best_f, return_scores=True)
    finally:
        engine.set_option("sweep_fused", 1)
    return mu.cpu().numpy(), var.cpu().numpy(), int(bi.item()), sg.cpu().numpy()


CASES = [
    # n, d, kind, m, acq
    (1, 1, "rbf", 1, "logei"),
    (2, 4, "rbf", 65, "ei"),
    (17, 5, "matern52", 1000, "logei"),
    (64, 8, "rbf", 4097, "logei"),
    (100, 3, "scale_linear_matern52", 777, "ucb"),
    (127, 16, "matern52", 2048, "variance"),
    (128, 8, "rbf", 3000, "ei"),
    (129, 4, "rbf", 5000, "logei"),
    (200, 13, "scale_linear_matern52", 1234, "logei"),
    (255, 8, "matern52", 999, "ucb"),
    (256, 4, "rbf", 20000, "logei"),
    (256, 16, "rbf", 1500, "ei"),
    (257, 8, "rbf", 3001, "logei"),
    (300, 4, "matern52", 2500, "ei"),
    (384, 8, "scale_linear_matern52", 1800, "logei"),
    (384, 13, "rbf", 700, "ucb"),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_fused_small_n_matches_oracle_and_unfused(engine, case):
    n, d, kind, m, acq = CASES[case]
    X, y = O.synthetic_problem(n, d, 50 + case)
    kp, op = pair(kind, d, noise=1e-4, outputscale=1.0 + 0.2 * case, const_mean=0.1)
    ost = O.fit(X, y, op)
    st = engine.fit(t(X), t(y), kp)
    Xs = O.sobol_candidates(m, d, case + 3) if m > 1 else np.random.default_rng(case).random((1, d))
    best_f = float(y.max())
    mu_f, var_f, bi_f, sg_f = _run(engine, st, Xs, acq, best_f, True)
    mu_u, var_u, bi_u, sg_u = _run(engine, st, Xs, acq, best_f, False)
    mu_r, var_r = O.posterior(ost, Xs)
    kdiag = O.kernel_diag(Xs, op)
    check_posterior(mu_f, var_f, mu_r.reshape(m, 1), var_r, kdiag)
    check_posterior(mu_f, var_f, mu_u, var_u, kdiag)
    _, _, sref = O.acquire_argmax(ost, Xs, ACQS[acq], best_f=best_f)
    check_argmax(bi_f, sref, sg_f, f"fused case {case}")
    check_argmax(bi_f, sg_u, sg_f, f"fused vs unfused case {case}")


def test_fused_sweep_nan_candidates_never_win(engine):
    n, d, m = 150, 6, 3000
    X, y = O.synthetic_problem(n, d, 5)
    kp, op = pair("rbf", d, noise=1e-4)
    st = engine.fit(t(X), t(y), kp)
    Xs = O.sobol_candidates(m, d, 9)
    Xs[[0, 17, 2999]] = np.nan
    mu_f, var_f, bi_f, sg_f = _run(engine, st, Xs, "logei", float(y.max()), True)
    _, _, bi_u, sg_u = _run(engine, st, Xs, "logei", float(y.max()), False)
    assert bi_f not in (0, 17, 2999)
    ok = ~np.isnan(Xs).any(axis=1)
    np.testing.assert_allclose(sg_f[ok], sg_u[ok], rtol=1e-9, atol=1e-12)
    assert bi_f == bi_u


@pytest.mark.parametrize("n,d,nrhs,kind", [(60, 5, 8, "rbf"), (200, 8, 3, "matern52"), (256, 16, 2, "scale_linear_matern52")])
def test_fused_multi_output_posterior(engine, n, d, nrhs, kind):
    """Multi-output posterior (Bayesian2.predict's 8 outputs sharing X): per-output means from the fused kernel."""
    X, y = O.synthetic_problem(n, d, n + nrhs)
    Y = np.stack([y * (r + 1) - 0.3 * r for r in range(nrhs)], axis=1)
    kp, op = pair(kind, d, noise=1e-4, const_mean=0.2)
    ost = O.fit(X, Y, op)
    st = engine.fit(t(X), t(Y), kp)
    Xs = O.sobol_candidates(3000, d, n)
    out = {}
    for fused in (True, False):
        engine.set_option("sweep_fused", 1 if fused else 0)
        try:
            mu, var = engine.posterior(st, t(Xs))
        finally:
            engine.set_option("sweep_fused", 1)
        out[fused] = (mu.cpu().numpy(), var.cpu().numpy())
    mu_r, var_r = O.posterior(ost, Xs)
    kdiag = O.kernel_diag(Xs, op)
    check_posterior(out[True][0], out[True][1], mu_r.reshape(3000, nrhs), var_r, kdiag)
    check_posterior(out[True][0], out[True][1], out[False][0], out[False][1], kdiag)
