"""CPU tests of the oracle: closed-form known answers and the committed golden fixtures.

Parity is unpinned against GPyTorch/BoTorch (not installed, no reference goldens — SURVEY §8c); these tests
pin the oracle's restatement to closed forms and to its own committed outputs.
"""
import glob
import math
import os

import numpy as np
import pytest
from scipy import integrate
from scipy.stats import norm

from oracle import gp_oracle as O
from tests.conftest import GOLDEN


def params(kind=O.RBF, d=3, **kw):
    return O.KernelParams(kind, np.full(d, kw.pop("ls", 0.7)), **kw)


def test_kernel_values_closed_form():
    a = np.array([[0.1, 0.2, 0.3]])
    b = np.array([[0.4, 0.0, 0.5]])
    ls = np.array([0.5, 1.0, 2.0])
    r2 = ((a - b) / ls) ** 2
    r2 = r2.sum()
    p = O.KernelParams(O.RBF, ls, outputscale=2.0)
    assert O.kernel_matrix(a, b, p)[0, 0] == pytest.approx(2.0 * math.exp(-0.5 * r2), rel=1e-15)
    p = O.KernelParams(O.MATERN52, ls, outputscale=1.5)
    r = math.sqrt(r2)
    expect = 1.5 * (1 + math.sqrt(5) * r + 5 / 3 * r2) * math.exp(-math.sqrt(5) * r)
    assert O.kernel_matrix(a, b, p)[0, 0] == pytest.approx(expect, rel=1e-14)
    lv = np.array([0.1, 0.2, 0.3])
    p = O.KernelParams(O.SCALE_LINEAR_MATERN52, ls, outputscale=1.5, linear_variance=lv)
    lin = float((a * lv * b).sum())
    assert O.kernel_matrix(a, b, p)[0, 0] == pytest.approx(1.5 * (lin + expect / 1.5), rel=1e-14)
    assert O.kernel_diag(a, p)[0] == pytest.approx(1.5 * ((a * a * lv).sum() + 1.0), rel=1e-15)


def test_gram_symmetric_pd():
    X, _ = O.synthetic_problem(64, 4, 0)
    for kind in (O.RBF, O.MATERN52, O.SCALE_LINEAR_MATERN52):
        K = O.gram(X, params(kind, 4))
        assert np.array_equal(K, K.T)
        assert np.linalg.eigvalsh(K).min() > 0


def test_one_point_posterior_closed_form():
    x = np.array([[0.3, 0.6]])
    y = np.array([1.7])
    p = O.KernelParams(O.RBF, np.array([0.4, 0.8]), outputscale=1.3, noise=0.05, const_mean=0.2)
    st = O.fit(x, y, p)
    xs = np.array([[0.5, 0.1], [0.3, 0.6]])
    k = O.kernel_matrix(xs, x, p)[:, 0]
    mu, var = O.posterior(st, xs)
    np.testing.assert_allclose(mu, 0.2 + k * (1.7 - 0.2) / (1.3 + 0.05), rtol=1e-14)
    np.testing.assert_allclose(var, 1.3 - k * k / (1.3 + 0.05), rtol=1e-13)


def test_noise_free_interpolation_and_floor():
    X, y = O.synthetic_problem(40, 2, 3)
    p = params(O.MATERN52, 2, noise=1e-12, ls=0.3)
    st = O.fit(X, y, p)
    mu, var = O.posterior(st, X)
    np.testing.assert_allclose(mu, y, atol=1e-6)
    assert var.min() >= O.GPYTORCH_MIN_VAR_F64  # gpytorch float64 floor then botorch floor
    assert np.all(var <= 1e-6)


def test_standardize_untransform():
    X, y = O.synthetic_problem(30, 3, 1)
    p = params(O.RBF, 3)
    st = O.fit(X, y, p)
    xs = O.sobol_candidates(16, 3, 2)
    mu0, var0 = O.posterior(st, xs)
    mu1, var1 = O.posterior(st, xs, y_mean=3.0, y_scale=2.0)
    np.testing.assert_allclose(mu1, 3.0 + 2.0 * mu0, rtol=1e-15)
    np.testing.assert_allclose(var1, 4.0 * var0, rtol=1e-15)


@pytest.mark.parametrize("u", [-30.0, -5.0, -1.5, -1.0, -0.3, 0.0, 0.7, 3.0])
def test_ei_matches_integral(u):
    # EI(u) with sigma=1 = E[max(Z - (-u), 0)] = int_{-u}^inf (z+u) phi(z) dz
    val, _ = integrate.quad(lambda z: (z + u) * norm.pdf(z), -u, np.inf, epsabs=1e-300, epsrel=1e-12)
    got = O.ei_helper(np.array([u]))[0]
    if val > 1e-250:
        assert got == pytest.approx(val, rel=1e-7, abs=1e-300)
        assert O.log_ei_helper(np.array([u]))[0] == pytest.approx(math.log(val), rel=1e-7, abs=1e-9)


def test_log_ei_branches_continuous_and_asymptotic():
    u = np.array([-1.0 - 1e-12, -1.0, -1.0 + 1e-12])
    v = O.log_ei_helper(u)
    assert np.all(np.abs(np.diff(v)) < 1e-10)
    # deep tail: log EI ~ -u^2/2 - log(sqrt(2pi)) - 2 log|u|
    uu = np.array([-1e8, -1e9])
    np.testing.assert_allclose(O.log_ei_helper(uu), -0.5 * uu * uu - 0.5 * math.log(2 * math.pi) - 2 * np.log(-uu),
                               rtol=1e-12)
    # moderate tail: log EI matches log of the direct EI where EI is still representable
    ul = np.linspace(-30, -1.01, 50)
    np.testing.assert_allclose(O.log_ei_helper(ul), np.log(O.ei_helper(ul)), rtol=1e-6)


def test_acquisition_forms():
    mu = np.array([0.1, 0.5, -1.0])
    var = np.array([0.04, 0.25, 1.0])
    s = np.sqrt(var)
    best = 0.3
    np.testing.assert_allclose(O.acquisition(mu, var, O.ACQ_UCB, beta=4.0), mu + 2.0 * s, rtol=1e-15)
    ei = O.acquisition(mu, var, O.ACQ_EI, best_f=best)
    np.testing.assert_allclose(ei, s * O.ei_helper((mu - best) / s), rtol=1e-15)
    np.testing.assert_allclose(O.acquisition(mu, var, O.ACQ_LOGEI, best_f=best), np.log(ei), rtol=1e-10)
    np.testing.assert_array_equal(O.acquisition(mu, var, O.ACQ_VARIANCE), var)


def test_argmax_lowest_index_and_nan():
    assert O.argmax_lowest(np.array([1.0, 3.0, 3.0, 2.0])) == (3.0, 1)
    assert O.argmax_lowest(np.array([np.nan, 1.0, np.nan, 1.0])) == (1.0, 1)
    assert O.combine_argmax([(2.0, 7), (2.0, 3), (1.0, 0), (np.nan, 1)]) == (2.0, 3)


def test_not_pd_pivot():
    X = np.array([[0.1, 0.2], [0.1, 0.2], [0.5, 0.5]])  # duplicate row
    p = params(O.RBF, 2, noise=0.0)
    with pytest.raises(O.NotPDError) as e:
        O.cholesky(O.gram(X, p))
    assert e.value.pivot == 1


def test_log_standardize_inputs_matches_bayesian7_definition():
    bounds = np.array([(0.3, 1.0), (0.001, 300.0), (0.001, 400.0), (2.0, 7.0), (2.0, 7.0)])
    Xu = O.sobol_candidates(64, 5, 4)
    Xs, m, s = O.log_standardize_inputs(Xu, bounds)
    Xp = Xu * (bounds[:, 1] - bounds[:, 0]) + bounds[:, 0]
    L = np.log(np.maximum(Xp, 1e-6))
    np.testing.assert_allclose(Xs, (L - L.mean(0)) / L.std(0, ddof=1), rtol=1e-13)


# oracle-output fixtures (the results_* / validation_* files are reference INPUTS, tests/test_gpu_realdata.py)
FIXTURES = sorted(f for f in glob.glob(os.path.join(GOLDEN, "*.npz"))
                  if not os.path.basename(f).startswith(("results_", "validation_")))


def _fixture_params(z):
    return O.KernelParams(int(z["kind"]), z["lengthscale"], outputscale=float(z["outputscale"]),
                          noise=float(z["noise"]), const_mean=float(z["const_mean"]),
                          linear_variance=z["linear_variance"], jitter=float(z["jitter"]))


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(f) for f in FIXTURES])
def test_oracle_reproduces_golden(path):
    z = np.load(path)
    p = _fixture_params(z)
    st = O.fit(z["X"], z["Y"], p)
    mu, var = O.posterior(st, z["Xs"])
    np.testing.assert_allclose(mu.reshape(z["mu"].shape), z["mu"], rtol=0, atol=1e-12 * np.abs(z["mu"]).max())
    np.testing.assert_allclose(var, z["var"], rtol=0, atol=1e-13)
    st0 = O.fit(z["X"], z["Y"][:, 0], p)
    for acq, aid in [("ei", O.ACQ_EI), ("logei", O.ACQ_LOGEI), ("ucb", O.ACQ_UCB), ("variance", O.ACQ_VARIANCE)]:
        v, i, _ = O.acquire_argmax(st0, z["Xs"], aid, best_f=float(z["best_f"]), beta=float(z["beta"]))
        assert i == int(z[f"argmax_{acq}"])


def test_reference_results_fixtures():
    """The full-size reference data of tests/test_gpu_realdata.py: row counts of the five results files (one corrupt row
    of optimization_results2.csv dropped), the 1550 duplicate X rows of optimization_results1009.csv, the validation
    rows, and the oracle's jitter choice on the duplicate file's head (noise-free: fails at jitter 0, taken at 1e-4)."""
    rows = {"r3000": (3000, 2), "r3901": (3901, 0), "r4235": (4235, 7), "r5000": (5000, 0), "r7740": (7740, 1550),
            "r2905": (2905, 0), "r173": (173, 2)}
    for tag, (n, dup) in rows.items():
        z = np.load(os.path.join(GOLDEN, f"results_{tag}.npz"))
        assert z["X"].shape == (n, 5) and z["Y"].shape == (n, 8) and int(z["duplicate_rows"]) == dup, tag
        assert np.isfinite(z["X"]).all() and np.isfinite(z["Y"]).all() and (z["Y"] > 0).all()
    assert list(np.load(os.path.join(GOLDEN, "results_r5000.npz"))["dropped"]) == [2384]
    assert np.load(os.path.join(GOLDEN, "validation_2048.npz"))["X"].shape == (2048, 5)
    assert O.psd_safe_jitters() == [0.0, 1e-4, 1e-3, 1e-2, 1e-1, 1.0]
    z = np.load(os.path.join(GOLDEN, "results_r7740.npz"))
    lo, hi = np.array([0.3, 0.001, 0.001, 2.0, 2.0]), np.array([1.0, 300.0, 400.0, 7.0, 7.0])
    Xu = (z["X"][:400] - lo) / (hi - lo)
    p = O.KernelParams(O.SCALE_LINEAR_MATERN52, np.full(5, 0.4), outputscale=1.5, noise=0.0,
                       linear_variance=np.linspace(0.05, 0.45, 5))
    st, jit, failed = O.fit_with_jitter(Xu, np.log(z["Y"][:400]), p)
    assert jit == 1e-4 and len(failed) == 1


def test_golden_fixtures_present():
    names = {os.path.basename(f) for f in FIXTURES}
    assert "real_b6_results256_val512.npz" in names and "real_b7_results256_val512.npz" in names
    assert len(FIXTURES) >= 7


@pytest.mark.parametrize("kind", [O.RBF, O.MATERN52, O.SCALE_LINEAR_MATERN52])
@pytest.mark.parametrize("n_old,q", [(1, 1), (40, 7), (100, 60)])
def test_append_equals_refit(kind, n_old, q):
    X, y = O.synthetic_problem(n_old + q, 4, n_old + q)
    Y = np.stack([y, 2 * y - 1], axis=1)
    p = params(kind, 4, noise=1e-4, linear_variance=np.full(4, 0.3))
    st = O.fit(X[:n_old], Y[:n_old], p)
    app = O.append(st, X, Y)
    ref = O.fit(X, Y, p)
    np.testing.assert_allclose(app.L, ref.L, rtol=0, atol=1e-12)
    np.testing.assert_allclose(app.alpha, ref.alpha, rtol=1e-9, atol=1e-9 * np.abs(ref.alpha).max())


def test_append_not_pd_global_pivot():
    X, y = O.synthetic_problem(30, 3, 1)
    X = np.vstack([X, [[50.0, 50.0, 50.0]], [[50.0, 50.0, 50.0]]])  # far away: K21 = 0 exactly, then a duplicate
    p = params(O.RBF, 3, noise=0.0, ls=0.5)
    st = O.fit(X[:30], y, params(O.RBF, 3, noise=0.0, ls=0.5))
    with pytest.raises(O.NotPDError) as e:
        O.append(st, X, np.zeros(32))
    assert e.value.pivot == 31


@pytest.mark.parametrize("kind,n,d,noise", [(O.RBF, 600, 8, 1e-4), (O.MATERN52, 600, 8, 1e-4), (O.RBF, 400, 4, 1e-6)])
def test_distance_form_gap_to_gpytorch_is_below_the_parity_tolerance(kind, n, d, noise):
    """The GPU kernels evaluate distances in the difference form sum_k ((a_k - b_k)/l_k)^2; GPyTorch [upstream] uses
    ||a||^2 + ||b||^2 - 2 a.b on mean-centred inputs.  Both are restated in the oracle (KernelParams.dist_form); this
    bounds how far the two formulations' posteriors drift apart on the north star's inputs, so that the 1e-9 parity
    tolerance against the oracle also bounds the distance to GPyTorch's arithmetic."""
    X, y = O.synthetic_problem(n, d, 5)
    ls = np.full(d, O.botorch_default_lengthscale(d))
    pd = O.KernelParams(kind, ls, noise=noise)
    pe = O.KernelParams(kind, ls, noise=noise, dist_form="expanded")
    Kd, Ke = O.gram(X, pd), O.gram(X, pe)
    assert np.abs(Kd - Ke).max() <= 1e-14  # O(eps) per entry
    Xs = O.sobol_candidates(500, d, 6)
    mu_d, var_d = O.posterior(O.fit(X, y, pd), Xs)
    mu_e, var_e = O.posterior(O.fit(X, y, pe), Xs)
    dmu = np.abs(mu_d - mu_e).max() / np.abs(mu_d).max()
    dvar = np.abs(var_d - var_e).max()
    assert dmu <= 1e-10, dmu
    assert dvar <= 1e-10, dvar
