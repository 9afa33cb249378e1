"""CPU tests of the host-side logic: parameter marshalling, transforms, sharding, and the drop-in optimizer
driven through run_optimization's call sequence (BASELINE configs[0]) with the oracle injected as engine."""
import math
import os

import numpy as np
import pytest
import torch

from bayesianoptimizer_amd import KernelParams, botorch_default_lengthscale
from bayesianoptimizer_amd.dist import combine_records_host, shard_range
from bayesianoptimizer_amd.models import ExactGP, LogExpectedImprovement, UpperConfidenceBound
from bayesianoptimizer_amd.optimizer import BayesianOptimizer, GPConfig, farthest_point_sampling
from bayesianoptimizer_amd.transforms import (LogInputStandardizer, LogOutputStandardizer, Standardize, normalize,
                                              unnormalize)
from oracle import gp_oracle as O
from tests.oracle_engine import OracleEngine
from tests.stubs import BOUNDS, StubSimulator, run_optimization_like


def test_kernel_params_to_c():
    p = KernelParams("scale_linear_matern52", [0.5, 0.6, 0.7], outputscale=2.0, noise=1e-3, jitter=1e-6,
                     const_mean=0.25, linear_variance=0.3)
    c = p.to_c(3)
    assert c.kind == 2 and c.d == 3
    assert list(c.lengthscale[:3]) == [0.5, 0.6, 0.7]
    assert list(c.linear_variance[:3]) == [0.3, 0.3, 0.3]
    assert (c.outputscale, c.noise, c.jitter, c.const_mean) == (2.0, 1e-3, 1e-6, 0.25)
    with pytest.raises(ValueError):
        KernelParams("rbf", [1.0, 2.0]).to_c(3)
    with pytest.raises(ValueError):
        KernelParams("nope").to_c(2)
    with pytest.raises(ValueError):
        KernelParams().to_c(33)


def test_default_lengthscale():
    assert botorch_default_lengthscale(8) == pytest.approx(0.5792, abs=1e-4)
    assert botorch_default_lengthscale(8) == pytest.approx(O.botorch_default_lengthscale(8), rel=1e-15)


def test_transforms():
    b = torch.tensor(BOUNDS, dtype=torch.float64).T
    g = torch.Generator().manual_seed(0)
    x = torch.rand(20, 5, dtype=torch.float64, generator=g)
    torch.testing.assert_close(normalize(unnormalize(x, b), b), x)
    xs = LogInputStandardizer(b).fit(x)(x)
    ref, _, _ = O.log_standardize_inputs(x.numpy(), np.array(BOUNDS))
    np.testing.assert_allclose(xs.numpy(), ref, rtol=1e-12, atol=1e-12)  # standardised values can sit near 0
    Y = torch.rand(20, 8, dtype=torch.float64) + 0.1
    tf = LogOutputStandardizer().fit(Y)
    torch.testing.assert_close(tf.inverse_mean(tf(Y)), Y)
    st = Standardize().fit(Y)
    torch.testing.assert_close(st.untransform_mean(st.transform(Y)), Y)


def test_shard_range_partitions():
    for total in [0, 1, 7, 32, 33]:
        for world in [1, 2, 3, 8]:
            spans = [shard_range(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    assert shard_range(32, 3, 8) == (12, 16)


def test_combine_records_host_order():
    v, i = combine_records_host(torch.tensor([1.0, 3.0, float("nan"), 3.0]), torch.tensor([5, 9, 0, 2]))
    assert (v, i) == (3.0, 2)


def test_exact_gp_and_acquisition_with_oracle_engine():
    X, y = O.synthetic_problem(50, 3, 2)
    Y = np.stack([y, 2 * y + 1], 1)
    eng = OracleEngine()
    gp = ExactGP(X, Y, KernelParams("rbf", 0.4, noise=1e-4), outcome_transform=Standardize(), engine=eng).fit()
    xs = O.sobol_candidates(64, 3, 3)
    post = gp.posterior(xs)
    assert post.mean.shape == (64, 2) and post.variance.shape == (64, 2)
    # output 1 = 2*y + 1 exactly: its untransformed posterior is 2*mu0 + 1, variance 4*var0
    torch.testing.assert_close(post.mean[:, 1], 2 * post.mean[:, 0] + 1, rtol=1e-9, atol=1e-9)
    torch.testing.assert_close(post.variance[:, 1], 4 * post.variance[:, 0], rtol=1e-9, atol=1e-12)
    v, i = LogExpectedImprovement(gp, best_f=float(Y[:, 0].max())).sweep(xs)
    scores = LogExpectedImprovement(gp, best_f=float(Y[:, 0].max()))(xs)
    assert int(i) == int(torch.argmax(scores))
    v2, i2 = UpperConfidenceBound(gp, beta=4.0).sweep(xs)
    assert 0 <= int(i2) < 64


def test_jitter_retry_policy():
    X = np.array([[0.1, 0.2], [0.1, 0.2], [0.5, 0.5]])  # duplicate rows: K singular without noise
    y = np.array([0.0, 0.1, 1.0])
    gp = ExactGP(X, y, KernelParams("rbf", 0.5, noise=0.0), engine=OracleEngine()).fit()
    assert gp.jitter_used == 1e-4
    from bayesianoptimizer_amd import NotPositiveDefiniteError

    with pytest.raises(NotPositiveDefiniteError):
        ExactGP(X, y, KernelParams("rbf", 0.5, noise=0.0), engine=OracleEngine(), jitter_schedule=(0.0,)).fit()


def test_farthest_point_sampling_spreads():
    X = torch.tensor(O.sobol_candidates(256, 2, 0))
    S = farthest_point_sampling(X, 8, np.random.default_rng(0))
    assert S.shape == (8, 2)
    d = torch.cdist(S, S) + torch.eye(8) * 10
    assert float(d.min()) > 0.15


@pytest.mark.parametrize("acq", ["variance", "logei"])
def test_dropin_optimizer_driven_like_run_optimization(tmp_path, acq):
    out = tmp_path / "run"
    cfg = GPConfig(candidates_pool_size=512, acq_batch_size=8, raw_samples=512)
    best_params, best_value = run_optimization_like(BayesianOptimizer, total_evaluations=40, n_initial_points=24,
                                                    batch_size=8, output_dir=str(out), engine=OracleEngine(),
                                                    gp_config=cfg, acquisition=acq, seed=0)
    assert best_params.shape == (5,)
    for k, (lo, hi) in enumerate(BOUNDS):
        assert lo - 1e-9 <= best_params[k] <= hi + 1e-9
    lines = open(out / "optimization_results.csv").read().strip().splitlines()
    assert lines[0].startswith("n,eta,sigma_y,width,height,x_01")
    assert len(lines) - 1 == 40
    log = open(out / "validation_log.csv").read().strip().splitlines()
    assert len(log) >= 2
    # resume: a larger target adds exactly the missing points, no new LHS
    run_optimization_like(BayesianOptimizer, total_evaluations=48, n_initial_points=24, batch_size=8,
                          output_dir=str(out), engine=OracleEngine(), gp_config=cfg, acquisition=acq, seed=1)
    lines2 = open(out / "optimization_results.csv").read().strip().splitlines()
    assert len(lines2) - 1 == 48
    # objective default: minimise the sum of outputs (Bayesian7.py:597-613,724-727)
    data = np.loadtxt(out / "optimization_results.csv", delimiter=",", skiprows=1)
    assert best_value == pytest.approx(data[:40, 5:].sum(1).min(), rel=1e-6)


def test_dropin_optimizer_qlogei_mode(tmp_path):
    # acquisition="qlogei": optimize_acqf on MC qLogEI with q = batch_size (Bayesian.py:96-113), small settings
    cfg = GPConfig(mc_samples=64, num_restarts=2, acqf_raw_samples=32, batch_limit=2, maxiter=5,
                   fit_hyperparameters=False)
    best_params, _ = run_optimization_like(BayesianOptimizer, total_evaluations=20, n_initial_points=16, batch_size=2,
                                           output_dir=str(tmp_path / "q"), engine=OracleEngine(), gp_config=cfg,
                                           acquisition="qlogei", seed=0)
    assert best_params.shape == (5,)
    lines = open(tmp_path / "q" / "optimization_results.csv").read().strip().splitlines()
    assert len(lines) - 1 == 20


def test_dropin_predict_matches_oracle(tmp_path):
    sim = StubSimulator()
    opt = BayesianOptimizer(sim, BOUNDS, str(tmp_path), n_initial_points=30, n_batches=0, batch_size=4,
                            target_total=30, engine=OracleEngine(), seed=3)
    opt.optimize()
    opt.fit_gp_model()
    xq = np.array([[0.5, 100.0, 200.0, 4.0, 5.0], [0.8, 10.0, 50.0, 3.0, 2.5]])
    y = opt.predict(xq)
    assert y.shape == (2, 8) and np.all(np.isfinite(y))


def test_product_default_engine_requires_gpu(tmp_path):
    if torch.cuda.is_available():
        pytest.skip("GPU present: the default engine is valid here")
    with pytest.raises(Exception):
        BayesianOptimizer(StubSimulator(), BOUNDS, str(tmp_path), 4, 1, 2, target_total=8)
