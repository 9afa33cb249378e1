"""Seeded randomized GPU parity sweep: random sizes (n 1..3000 incl. non-multiples of 64/128, d 1..32), kernels,
output counts, noise levels and candidate counts, every case checked against the oracle at the parity tolerances of
tests/test_gpu_parity.py (posterior mean 1e-9 of max|mu|, variance 1e-9 of k(x,x), argmax exact or a reported tie)."""
import numpy as np
import pytest
import torch

from oracle import gp_oracle as O
from tests.test_gpu_parity import DEV, check_argmax, check_posterior, pair, t

pytestmark = pytest.mark.gpu
KINDS = ["rbf", "matern52", "scale_linear_matern52"]
ACQS = {"ei": O.ACQ_EI, "logei": O.ACQ_LOGEI, "ucb": O.ACQ_UCB, "variance": O.ACQ_VARIANCE}


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.choice([1, 2, 63, 64, 65, 127, 129, 255, 300, 511, 777, 1025, 1500, 2049, 3000]))
    d = int(rng.choice([1, 2, 3, 5, 8, 13, 16, 31, 32]))
    kind = KINDS[seed % 3]
    nrhs = int(rng.integers(1, 9))
    noise = float(10.0 ** rng.uniform(-5, -1))
    ls = float(np.sqrt(d) * 10.0 ** rng.uniform(-0.6, 0.2))
    m = int(rng.choice([1, 7, 256, 1000, 5000]))
    acq = list(ACQS)[seed % 4]
    return n, d, kind, nrhs, noise, ls, m, acq


@pytest.mark.parametrize("seed", range(36))
def test_random_fit_posterior_acquire(engine, seed):
    n, d, kind, nrhs, noise, ls, m, acq = _case(seed)
    X, y = O.synthetic_problem(n, d, seed)
    Y = np.stack([y * (r + 1) - 0.5 * r for r in range(nrhs)], axis=1)
    kp, op = pair(kind, d, ls=ls, noise=noise, outputscale=1.0 + 0.1 * (seed % 5), const_mean=0.05 * (seed % 3))
    try:
        ost = O.fit(X, Y, op)
    except O.NotPDError:
        pytest.skip("oracle Gram not positive definite for this draw")
    st = engine.fit(t(X), t(Y), kp)
    Xs = O.sobol_candidates(m, d, seed + 7) if m > 1 else np.random.default_rng(seed).random((1, d))
    mu, var = engine.posterior(st, t(Xs))
    mu_r, var_r = O.posterior(ost, Xs)
    check_posterior(mu.cpu().numpy(), var.cpu().numpy(), mu_r.reshape(m, nrhs), var_r, O.kernel_diag(Xs, op))
    best_f = float(Y[:, 0].max())
    bv, bi, sg = engine.acquire(st, t(Xs), acq, best_f=best_f, return_scores=True)
    ost1 = O.GPState(ost.X, ost.L, ost.alpha.reshape(n, nrhs)[:, 0], op)
    _, _, sref = O.acquire_argmax(ost1, Xs, ACQS[acq], best_f=best_f)
    check_argmax(int(bi.item()), sref, sg.cpu().numpy(), f"case {seed}")
