"""CPU tests of the host side of the optimize_acqf refinement: the oracle's gradient restatement
(finite differences), the smooth maths and MC reduction in torch against the oracle, the Sobol base samples and the
Boltzmann restart selection.  The GPU posterior-gradient kernel is covered in tests/test_acqf.py."""
import numpy as np
import pytest
import torch

from bayesianoptimizer_amd import acqf
from oracle import gp_oracle as O


@pytest.mark.parametrize("kind", [O.RBF, O.MATERN52, O.SCALE_LINEAR_MATERN52])
def test_oracle_moment_gradients_match_finite_differences(kind):
    X, y = O.synthetic_problem(40, 3, 2)
    p = O.KernelParams(kind, np.full(3, 0.5), linear_variance=np.full(3, 0.3), noise=1e-3, outputscale=1.2)
    st = O.fit(X, y, p)
    Xs = np.random.default_rng(0).random((6, 3))
    mean, dmean, cov, dcov = O.moments_grad(st, Xs, 3)
    h = 1e-6
    for a in range(6):
        for j in range(3):
            Xp, Xm = Xs.copy(), Xs.copy()
            Xp[a, j] += h
            Xm[a, j] -= h
            mp, _, cp, _ = O.moments_grad(st, Xp, 3)
            mm, _, cm, _ = O.moments_grad(st, Xm, 3)
            assert abs((mp[a] - mm[a]) / (2 * h) - dmean[a, j]) < 1e-6
            b0 = (a // 3) * 3
            for c in range(3):
                total = dcov[a, j, c] * (2 if b0 + c == a else 1)  # diagonal: both arguments move
                assert abs((cp[a, c] - cm[a, c]) / (2 * h) - total) < 1e-6


def test_log_ei_helper_matches_oracle():
    u = np.concatenate([np.linspace(-50, 10, 601), [-1.0, -1e4, -1e9]])
    got = acqf.log_ei_helper(torch.tensor(u)).numpy()
    np.testing.assert_allclose(got, O.log_ei_helper(u), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("fat", [True, False])
@pytest.mark.parametrize("q", [1, 3])
def test_qlogei_reduction_matches_oracle(fat, q):
    rng = np.random.default_rng(q)
    B = 4
    mu = rng.standard_normal((B, q))
    A = rng.standard_normal((B, q, q))
    Sigma = A @ np.swapaxes(A, 1, 2) * 0.1 + 0.01 * np.eye(q)
    z = O.sobol_normal_base_samples(256, q, seed=5)
    sampler = acqf.SobolQMCNormalSampler(torch.Size([256]), seed=5)
    np.testing.assert_allclose(sampler.base_samples(q, "cpu").numpy(), z, rtol=0, atol=1e-14)  # erfinv ulps
    for best_f in (-1.0, 0.5, 3.0):  # far above the mean: the log-improvement tail branch
        got = acqf.qlogei_from_moments(torch.tensor(mu), torch.tensor(Sigma), torch.tensor(z), best_f, fat).numpy()
        ref = O.qlogei(mu, Sigma, z, best_f, fat)
        np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-10)


def test_sobol_base_samples_are_standard_normal_and_seeded():
    a = acqf.SobolQMCNormalSampler(torch.Size([1024]), seed=3).base_samples(2, "cpu")
    b = acqf.SobolQMCNormalSampler(torch.Size([1024]), seed=3).base_samples(2, "cpu")
    assert torch.equal(a, b)
    assert abs(float(a.mean())) < 0.02 and abs(float(a.std()) - 1.0) < 0.02


def test_initialize_q_batch_keeps_best_and_is_seeded():
    X = torch.arange(200, dtype=torch.float64).view(100, 1, 2)
    Y = torch.linspace(0, 1, 100, dtype=torch.float64)
    Y[37] = 5.0
    g1, g2 = torch.Generator().manual_seed(1), torch.Generator().manual_seed(1)
    a = acqf.initialize_q_batch(X, Y, 10, generator=g1)
    b = acqf.initialize_q_batch(X, Y, 10, generator=g2)
    assert torch.equal(a, b)
    assert any(torch.equal(r, X[37]) for r in a)
    assert acqf.initialize_q_batch(X, Y, 100) is X
    const = acqf.initialize_q_batch(X, torch.zeros(100, dtype=torch.float64), 5, generator=g1)
    assert const.shape == (5, 1, 2)
    with pytest.raises(ValueError):
        acqf.initialize_q_batch(X, Y, 101)


def test_psd_safe_cholesky_jitter():
    S = torch.tensor([[[1.0, 1.0], [1.0, 1.0]]], dtype=torch.float64)  # singular: needs the jitter
    L = acqf.psd_safe_cholesky(S)
    assert torch.allclose(L @ L.transpose(1, 2), S, atol=1e-6)
