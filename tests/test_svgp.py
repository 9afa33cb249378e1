"""Driven variant (optimization/Bayesian7.py): batched SVGP predictive, top-k and farthest point sampling.

CPU tests pin the oracle restatement (known answers) and the checkpoint loader; GPU tests compare the HIP path
(gpx_svgp_*, gpx_topk_f64, gpx_fps_f64) with the oracle on identical inputs:
  SVGP mean |d mu| <= 1e-9 max|mu|, variance |d var| <= 1e-9 max var (fp64 both sides);
  top-k and FPS indices bit-exact (ties -> lowest index, documented deterministic order).
"""
import numpy as np
import pytest
import torch

from bayesianoptimizer_amd import KernelParams
from bayesianoptimizer_amd.svgp import NOISE_LOWER_BOUND, SVGPModel
from oracle import gp_oracle as O


def svgp_problem(T=3, M=300, d=5, seed=0):
    rng = np.random.default_rng(seed)
    Z = rng.standard_normal((T, M, d))
    vmean = rng.standard_normal((T, M))
    vchol = np.tril(0.3 * rng.standard_normal((T, M, M)) / np.sqrt(M))
    for t in range(T):
        vchol[t][np.diag_indices(M)] = 0.2 + 0.5 * rng.random(M)
    vchol += np.triu(rng.standard_normal((T, M, M)), 1)  # garbage above the diagonal must be ignored
    kps, ops = [], []
    for t in range(T):
        ls = 0.8 + rng.random(d)
        lv = 0.05 + 0.1 * rng.random(d)
        os_, noise, c = 0.5 + rng.random(), 1e-3 * (t + 1), 0.1 * t - 0.2
        kps.append(KernelParams("scale_linear_matern52", list(ls), outputscale=os_, noise=noise, const_mean=c,
                                linear_variance=list(lv)))
        ops.append(O.KernelParams(O.SCALE_LINEAR_MATERN52, ls, outputscale=os_, noise=noise, const_mean=c,
                                  linear_variance=lv))
    return Z, vmean, vchol, kps, ops


# ---- CPU: oracle known answers and the checkpoint loader ----------------------------------------------------
def test_oracle_svgp_prior_and_noiseless_limits():
    Z, vmean, vchol, _, ops = svgp_problem(T=1, M=40, d=3, seed=1)
    Xs = np.random.default_rng(2).standard_normal((25, 3))
    # q(u) = prior (m = 0, S = I): predictive = prior mean / variance + noise
    mu, var, score = O.svgp_predict(Z, np.zeros((1, 40)), np.eye(40)[None], ops, Xs)
    np.testing.assert_allclose(mu[:, 0], ops[0].const_mean, atol=1e-14)
    np.testing.assert_allclose(var[:, 0], O.kernel_diag(Xs, ops[0]) + ops[0].noise, rtol=1e-12)
    np.testing.assert_allclose(score, var.sum(1))
    # S = 0: k** - k*^T (K_ZZ + jitter I)^{-1} k* + noise
    mu0, var0, _ = O.svgp_predict(Z, vmean, np.zeros((1, 40, 40)), ops, Xs)
    Kzz = O.kernel_matrix(Z[0], Z[0], ops[0]) + O.VARIATIONAL_JITTER_F32 * np.eye(40)
    Kzx = O.kernel_matrix(Z[0], Xs, ops[0])
    ref = O.kernel_diag(Xs, ops[0]) - np.einsum("ij,ij->j", Kzx, np.linalg.solve(Kzz, Kzx)) + ops[0].noise
    np.testing.assert_allclose(var0[:, 0], ref, rtol=1e-9, atol=1e-12)
    # mean = c + k*^T L^{-T} m
    L = np.linalg.cholesky(Kzz)
    np.testing.assert_allclose(mu0[:, 0], ops[0].const_mean + Kzx.T @ np.linalg.solve(L.T, vmean[0]), rtol=1e-9,
                               atol=1e-12)


def test_oracle_topk_and_fps_known_answers():
    v, i = O.topk_desc(np.array([0.5, 2.0, np.nan, 2.0, -1.0, 2.0]), 4)
    assert list(i) == [1, 3, 5, 0] and list(v) == [2.0, 2.0, 2.0, 0.5]
    # points on a line: from 0 the farthest is the end, then the middle, then the quarter points (lowest index wins)
    X = np.linspace(0.0, 1.0, 9)[:, None]
    assert list(O.farthest_point_sampling(X, 5, 0)) == [0, 8, 4, 2, 6]
    # duplicates: once everything left is at distance 0 the lowest index is returned again (torch.argmax)
    X2 = np.array([[0.0], [1.0], [1.0], [0.0]])
    assert list(O.farthest_point_sampling(X2, 4, 0)) == [0, 1, 0, 0]


def test_svgp_model_from_gpytorch_state_dict():
    T, M, d = 2, 7, 3
    g = torch.Generator().manual_seed(0)
    raw = lambda *s: torch.randn(*s, generator=g, dtype=torch.float32)  # noqa: E731
    sd = {
        "variational_strategy.inducing_points": raw(T, M, d),
        "variational_strategy._variational_distribution.variational_mean": raw(T, M),
        "variational_strategy._variational_distribution.chol_variational_covar": raw(T, M, M),
        "mean_module.raw_constant": raw(T),
        "covar_module.raw_outputscale": raw(T),
        "covar_module.base_kernel.kernels.0.raw_variance": raw(T, 1, d),
        "covar_module.base_kernel.kernels.1.raw_lengthscale": raw(T, 1, d),
    }
    lik = {"noise_covar.raw_noise": raw(T, 1)}
    m = SVGPModel.from_state_dict(sd, lik)
    sp = lambda x: torch.nn.functional.softplus(x.double())  # noqa: E731
    assert m.num_tasks == T and m.Z.dtype == torch.float64
    for t in range(T):
        p = m.params[t]
        assert p.kind == "scale_linear_matern52"
        np.testing.assert_allclose(p.lengthscale, sp(sd["covar_module.base_kernel.kernels.1.raw_lengthscale"][t, 0]))
        np.testing.assert_allclose(p.linear_variance, sp(sd["covar_module.base_kernel.kernels.0.raw_variance"][t, 0]))
        assert p.outputscale == pytest.approx(float(sp(sd["covar_module.raw_outputscale"][t])))
        assert p.noise == pytest.approx(float(sp(lik["noise_covar.raw_noise"][t, 0])) + NOISE_LOWER_BOUND)
        assert p.const_mean == pytest.approx(float(sd["mean_module.raw_constant"][t]))


# ---- GPU: the HIP path against the oracle ---------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("T,M,d,m", [(3, 300, 5, 700), (8, 128, 5, 2500), (1, 1000, 8, 300)])
def test_svgp_predict_matches_oracle(engine, T, M, d, m):
    Z, vmean, vchol, kps, ops = svgp_problem(T, M, d, seed=T + M)
    Xs = np.random.default_rng(9).standard_normal((m, d))
    prep = engine.svgp_prepare(kps, Z, vmean, vchol)
    mu, var, score = engine.svgp_predict(prep, torch.tensor(Xs, device=engine.device))
    mu_r, var_r, score_r = O.svgp_predict(Z, vmean, vchol, ops, Xs)
    mu, var, score = mu.cpu().numpy(), var.cpu().numpy(), score.cpu().numpy()
    assert np.abs(mu - mu_r).max() <= 1e-9 * np.abs(mu_r).max()
    assert np.abs(var - var_r).max() <= 1e-9 * np.abs(var_r).max()
    assert np.abs(score - score_r).max() <= 1e-9 * np.abs(score_r).max()


@pytest.mark.gpu
def test_topk_matches_oracle_with_ties_and_nan(engine):
    rng = np.random.default_rng(3)
    s = np.round(rng.random(20000) * 50) / 7.0  # many exact ties
    s[[5, 77, 1999]] = np.nan
    s[100] = -0.0
    s[101] = 0.0
    v, i = engine.topk(torch.tensor(s, device=engine.device), 15000)
    v_r, i_r = O.topk_desc(s, 15000)
    np.testing.assert_array_equal(i.cpu().numpy(), i_r)
    np.testing.assert_array_equal(v.cpu().numpy(), v_r)


@pytest.mark.gpu
@pytest.mark.parametrize("m,d,k,start", [(8000, 5, 500, 1234), (3000, 2, 300, 0), (20000, 8, 64, 19999),
                                         (9, 1, 5, 0),
                                         # the register-resident kernels' edges (gpx_svgp.hip launch_fps): 1024 x 8
                                         # points at d <= 4, 512 x 16 at d = 5, the re-reading kernel beyond
                                         (8192, 4, 200, 8191), (8192, 5, 200, 0), (8193, 5, 50, 8192),
                                         (1024, 6, 100, 7), (64, 3, 64, 5)])
def test_fps_matches_oracle(engine, m, d, k, start):
    X = np.random.default_rng(m + d).random((m, d))
    if m == 9:
        X = np.linspace(0.0, 1.0, 9)[:, None]
    idx = engine.fps(torch.tensor(X, device=engine.device), k, start).cpu().numpy()
    np.testing.assert_array_equal(idx, O.farthest_point_sampling(X, k, start))


@pytest.mark.gpu
def test_pool_scan_end_to_end(engine):
    """Bayesian7's acquisition block (:646-688) on a 10,000-candidate pool: score -> top K_big -> FPS."""
    from bayesianoptimizer_amd.svgp import SVGPPredictor

    T, M, d = 8, 256, 5
    Z, vmean, vchol, kps, ops = svgp_problem(T, M, d, seed=11)
    model = SVGPModel(Z=torch.tensor(Z), vmean=torch.tensor(vmean), vchol=torch.tensor(vchol), params=kps)
    pred = SVGPPredictor(model, engine)
    cand = np.random.default_rng(5).random((10000, d))
    pts, idx = pred.pool_scan(torch.tensor(cand), batch_k=300, start=42)
    _, _, score_r = O.svgp_predict(Z, vmean, vchol, ops, cand)
    k_big = min(max(5000, 20 * 300), 8000, 10000)
    _, big = O.topk_desc(score_r, k_big)
    sel = O.farthest_point_sampling(cand[big], 300, 42)
    np.testing.assert_array_equal(idx.cpu().numpy(), big[sel])
    np.testing.assert_array_equal(pts.cpu().numpy(), cand[big[sel]])


@pytest.mark.gpu
def test_svgp_driven_config_T8_M2048_pool_scan(engine):
    """The configuration Bayesian7 actually runs (/root/reference/optimization/Bayesian7.py:32,45,57,63,138): T = 8
    tasks, M = 2048 inducing points, a 10,000-candidate LHS pool scored in 2048-row chunks, top K_big = 8000 by the
    variance sum, then farthest-point sampling of acq_batch_size = 500.  Predictive mean / variance / score against the
    oracle at 1e-9 and the selected pool indices bit-exact against the oracle's top-k + FPS on the oracle's scores."""
    from bayesianoptimizer_amd.svgp import SVGPPredictor

    T, M, d, m, batch_k = 8, 2048, 5, 10000, 500
    Z, vmean, vchol, kps, ops = svgp_problem(T, M, d, seed=2048)
    cand = np.random.default_rng(6).random((m, d))
    model = SVGPModel(Z=torch.tensor(Z), vmean=torch.tensor(vmean), vchol=torch.tensor(vchol), params=kps)
    pred = SVGPPredictor(model, engine)
    mu, var, score = engine.svgp_predict(pred.prep, torch.tensor(cand, device=engine.device))
    mu_r, var_r, score_r = O.svgp_predict(Z, vmean, vchol, ops, cand)
    mu, var, score = mu.cpu().numpy(), var.cpu().numpy(), score.cpu().numpy()
    assert np.abs(mu - mu_r).max() <= 1e-9 * np.abs(mu_r).max()
    assert np.abs(var - var_r).max() <= 1e-9 * np.abs(var_r).max()
    assert np.abs(score - score_r).max() <= 1e-9 * np.abs(score_r).max()
    pts, idx = pred.pool_scan(torch.tensor(cand), batch_k=batch_k, start=123)
    k_big = min(max(5000, 20 * batch_k), 8000, m)
    _, big = O.topk_desc(score_r, k_big)
    sel = O.farthest_point_sampling(cand[big], batch_k, 123)
    np.testing.assert_array_equal(idx.cpu().numpy(), big[sel])
