"""The drop-in optimizer driven exactly like scripts/run_optimization.py:116-133 on the real HIP engine:
every acquisition mode end to end on the GPU, and the GPU run's GP agreeing with the oracle-engine run's GP."""
import numpy as np
import pytest
import torch

from bayesianoptimizer_amd.optimizer import BayesianOptimizer, GPConfig
from tests.oracle_engine import OracleEngine
from tests.stubs import BOUNDS, StubSimulator, run_optimization_like

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("acq", ["variance", "logei", "qlogei"])
def test_dropin_on_gpu(tmp_path, engine, acq):
    cfg = GPConfig(candidates_pool_size=2048, raw_samples=1024, mc_samples=128, num_restarts=4, acqf_raw_samples=128,
                   batch_limit=2, maxiter=30)
    best_params, best_value = run_optimization_like(BayesianOptimizer, total_evaluations=48, n_initial_points=32,
                                                    batch_size=4, output_dir=str(tmp_path / acq), engine=engine,
                                                    gp_config=cfg, acquisition=acq, seed=0)
    assert best_params.shape == (5,) and np.isfinite(best_value)
    for k, (lo, hi) in enumerate(BOUNDS):
        assert lo - 1e-9 <= best_params[k] <= hi + 1e-9
    data = np.loadtxt(tmp_path / acq / "optimization_results.csv", delimiter=",", skiprows=1)
    assert data.shape[0] == 48
    assert best_value == pytest.approx(data[:, 5:].sum(1).min(), rel=1e-6)


def test_dropin_gpu_model_matches_oracle_engine(tmp_path, engine):
    # fixed hyperparameters: the same posterior on both engines (with fitting, L-BFGS-B trajectories on a
    # non-convex marginal likelihood may part at the 1e-9 level of the objectives and end in different optima)
    cfg = GPConfig(fit_hyperparameters=False)
    sims = []
    opts = []
    for eng, name in ((engine, "gpu"), (OracleEngine(), "cpu")):
        sim = StubSimulator()
        opt = BayesianOptimizer(sim, BOUNDS, str(tmp_path / name), n_initial_points=40, n_batches=0, batch_size=4,
                                target_total=40, engine=eng, gp_config=cfg, seed=3)
        opt.optimize()
        opt.fit_gp_model()
        sims.append(sim)
        opts.append(opt)
    xq = np.array([[0.5, 100.0, 200.0, 4.0, 5.0], [0.8, 10.0, 50.0, 3.0, 2.5], [0.3, 500.0, 20.0, 6.0, 7.0]])
    y_gpu, y_cpu = opts[0].predict(xq), opts[1].predict(xq)
    np.testing.assert_allclose(y_gpu, y_cpu, rtol=1e-8, atol=1e-10)
    for s in sims:
        s.cleanup()


def test_dropin_crosses_svgp_threshold_on_gpu(tmp_path, engine):
    """The driver's threshold (scripts/run_optimization.py:40: 3000), with the opt-in large-n policy: below it the GP is
    refitted by marginal
    likelihood each round, above it hyperparameters come from a 3000-point subsample, the exact posterior covers every
    point, and later rounds use the bordered update; the posterior then equals a fresh fit on the same data."""
    from bayesianoptimizer_amd.models import ExactGP
    from oracle import gp_oracle as O

    cfg = GPConfig(candidates_pool_size=2048, acq_batch_size=20, fit_hyperparameters=True, prior_set="none",
                   mll_options={"maxiter": 15}, large_n_policy=True)
    opt = BayesianOptimizer(StubSimulator(), BOUNDS, str(tmp_path), n_initial_points=2990, n_batches=3, batch_size=20,
                            svgp_threshold=3000, target_total=3050, engine=engine, gp_config=cfg, seed=1)
    opt.optimize()
    opt.fit_gp_model()
    gp = opt.gp_model
    assert opt.train_X.shape[0] == 3050
    assert opt._large_n_base == 3010          # the first round above the threshold rebuilt the factor
    assert gp.independent                      # hyperparameters per output (the multi-output SingleTaskGP)
    assert all(st.n == 3050 for st in gp.states)  # the rows since were folded in by the bordered update, per output
    assert len({tuple(p.lengthscales(5)) for p in gp.params}) > 1
    ref = ExactGP(gp.train_X, opt.y_tf(opt.train_Y_raw), gp.params, engine=engine).fit()
    Xq = opt.x_tf(torch.tensor(O.sobol_candidates(512, 5, 3), device=engine.device))
    a, b = gp.posterior(Xq), ref.posterior(Xq)
    scale = b.mean.abs().max()
    assert (a.mean - b.mean).abs().max() <= 1e-9 * scale
    # the parity scale of a variance is the prior variance k(x, x) >= outputscale, not the posterior
    # variance, which at 3050 points is ~1e-6 (bordered update vs refit measured 4.6e-12 absolute)
    os_min = min(p.outputscale for p in gp.params)
    assert (a.variance - b.variance).abs().max() <= 1e-9 * os_min


def test_dropin_survives_timed_out_handoffs(tmp_path, engine):
    """with spin_limit = 0 every in-launch hand-off of the persistent backward solve times out.
    ExactGP.fit then refits the same jitter through the hand-off-free inverse path (multi-launch TRTRI, alpha = W W^T y),
    so BayesianOptimizer.optimize() runs to completion (the reference's fit, optimization/Bayesian6.py:482-488, has no
    such failure mode) and the final model's alpha and posterior equal the oracle's."""
    from oracle import gp_oracle as O
    from tests.oracle_engine import to_oracle_params

    cfg = GPConfig(fit_hyperparameters=False, incremental_updates=False, raw_samples=4096)
    sim = StubSimulator()
    engine.set_option("spin_limit", 0)
    try:
        opt = BayesianOptimizer(sim, BOUNDS, str(tmp_path / "to"), n_initial_points=600, n_batches=2, batch_size=8,
                                target_total=616, engine=engine, gp_config=cfg, acquisition="logei", seed=5)
        best_params, best_value = opt.optimize()
        opt.fit_gp_model()
        gp = opt.gp_model
        assert gp.timeout_fallbacks >= 1  # 600+ points: 5+ row blocks, so the solve has hand-offs to time out
        X = gp.train_X.cpu().numpy()
        Y = gp.train_Y.cpu().numpy()
        a = gp.state.alpha[: X.shape[0]].cpu().numpy()
    finally:
        engine.set_option("spin_limit", 1 << 22)
        sim.cleanup()
    assert np.isfinite(best_value) and best_params.shape == (5,)
    data = np.loadtxt(tmp_path / "to" / "optimization_results.csv", delimiter=",", skiprows=1)
    assert data.shape[0] == 616
    ost = O.fit(X, Y, to_oracle_params(gp.params.replace(jitter=gp.jitter_used), X.shape[1]))
    ar = ost.alpha.reshape(a.shape)
    assert np.abs(a - ar).max() <= 1e-8 * np.abs(ar).max()
    Xq = np.random.default_rng(1).random((64, X.shape[1]))
    post = gp.posterior(torch.tensor(Xq, device=engine.device))
    mu_r, _ = O.posterior(ost, Xq)
    mu_r = mu_r.reshape(64, -1)
    assert gp.outcome_transform is None  # the drop-in standardises the targets itself (Bayesian7.py:363-385)
    mu = post.mean.cpu().numpy()
    assert np.abs(mu - mu_r).max() <= 1e-9 * np.abs(mu_r).max()
