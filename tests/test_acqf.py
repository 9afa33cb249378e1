"""GPU tests of the optimize_acqf refinement: gpx_moments_grad_f64 against the oracle's
restatement, the autograd chain rule against finite differences, the differentiable acquisition values against the
GPU sweep and the oracle's qLogEI, and optimize_acqf end to end."""
import numpy as np
import pytest
import torch

from bayesianoptimizer_amd import acqf
from bayesianoptimizer_amd.models import ExactGP
from bayesianoptimizer_amd.transforms import Standardize
from oracle import gp_oracle as O
from tests.test_gpu_parity import DEV, pair, t

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["rbf", "matern52", "scale_linear_matern52"])
@pytest.mark.parametrize("n,q,m", [(200, 1, 37), (700, 3, 30), (1500, 4, 64)])
def test_moments_grad_matches_oracle(engine, kind, n, q, m):
    d = 5
    X, y = O.synthetic_problem(n, d, n + q)
    kp, op = pair(kind, d, noise=1e-3, outputscale=1.4, const_mean=0.2)
    st = engine.fit(t(X), t(y), kp)
    ost = O.fit(X, y, op)
    Xs = np.random.default_rng(m).random((m, d))
    mean, dmean, cov, dcov = (v.cpu().numpy() for v in engine.moments_grad(st, t(Xs), q))
    rm, rdm, rc, rdc = O.moments_grad(ost, Xs, q)
    assert np.abs(mean - rm).max() <= 1e-9 * np.abs(rm).max()
    assert np.abs(dmean - rdm).max() <= 1e-8 * np.abs(rdm).max()
    assert np.abs(cov - rc).max() <= 1e-9 * op.outputscale
    assert np.abs(dcov - rdc).max() <= 1e-8 * np.abs(rdc).max()


def _model(n=400, d=4, kind="matern52", nrhs=1, seed=3):
    X, y = O.synthetic_problem(n, d, seed)
    Y = np.stack([y * (r + 1) + r for r in range(nrhs)], axis=1)
    kp, op = pair(kind, d, noise=1e-3)
    return ExactGP(X, Y, kp, outcome_transform=Standardize()).fit(), X, Y, op


def test_autograd_chain_rule_matches_finite_differences(engine):
    gp, X, Y, op = _model()
    rng = np.random.default_rng(0)
    Xq = torch.tensor(rng.random((3, 4, 4)), device=DEV, requires_grad=True)
    wm = torch.tensor(rng.standard_normal((3, 4)), device=DEV)
    wc = torch.tensor(rng.standard_normal((3, 4, 4)), device=DEV)

    def f(Z):
        mu, cov = acqf.posterior_moments(gp, Z)
        return (wm * mu).sum() + (wc * cov).sum()

    (g,) = torch.autograd.grad(f(Xq), Xq)
    h = 1e-6
    Xd = Xq.detach()
    fd = torch.zeros_like(Xd)
    for idx in np.ndindex(*Xd.shape):
        e = torch.zeros_like(Xd)
        e[idx] = h
        fd[idx] = (f(Xd + e) - f(Xd - e)) / (2 * h)
    assert (g - fd).abs().max().item() <= 1e-6 * max(1.0, fd.abs().max().item())


@pytest.mark.parametrize("kind", ["logei", "ei", "ucb"])
def test_analytic_values_match_sweep_and_gradient_fd(engine, kind):
    gp, X, Y, op = _model(nrhs=2)
    best_f = float(Y[:, 1].max())
    cls = {"logei": acqf.LogExpectedImprovement, "ei": acqf.ExpectedImprovement, "ucb": acqf.UpperConfidenceBound}[kind]
    a = cls(gp, best_f=best_f, output=1)
    Xc = torch.tensor(O.sobol_candidates(256, 4, 2), device=DEV)
    vals = a(Xc.unsqueeze(1))
    from bayesianoptimizer_amd.models import ExpectedImprovement, LogExpectedImprovement, UpperConfidenceBound

    sweep_cls = {"logei": LogExpectedImprovement, "ei": ExpectedImprovement, "ucb": UpperConfidenceBound}[kind]
    ref = sweep_cls(gp, best_f=best_f, output=1)(Xc)
    assert (vals - ref).abs().max().item() <= 1e-9 * max(1.0, ref.abs().max().item())
    Xg = Xc[:8].clone().unsqueeze(1).requires_grad_(True)
    (g,) = torch.autograd.grad(a(Xg).sum(), Xg)
    h = 1e-6
    for i in range(8):
        for j in range(4):
            e = torch.zeros_like(Xg)
            e[i, 0, j] = h
            with torch.no_grad():
                fd = (a(Xg + e).sum() - a(Xg - e).sum()) / (2 * h)
            assert abs(g[i, 0, j].item() - fd.item()) <= 1e-5 * max(1.0, abs(fd.item()))


@pytest.mark.parametrize("q,weights", [(1, None), (3, None), (2, [0.5, 0.5])])
def test_qlogei_matches_oracle(engine, q, weights):
    nrhs = 2 if weights else 1
    gp, X, Y, op = _model(nrhs=nrhs)
    w = np.array(weights) if weights else np.array([1.0])
    best_f = float((Y @ w).max())
    sampler = acqf.SobolQMCNormalSampler(torch.Size([256]), seed=11)
    obj = acqf.LinearMCObjective(weights) if weights else None
    a = acqf.qLogExpectedImprovement(gp, best_f=best_f, sampler=sampler, objective=obj)
    B = 6
    Xq = np.random.default_rng(q).random((B, q, 4))
    got = a(torch.tensor(Xq, device=DEV)).cpu().numpy()
    # oracle: joint posterior of the objective in original units from the standardized fit
    mean, std = Y.mean(0), Y.std(0, ddof=1)
    Ys = (Y - mean) / std
    ost = O.fit(X, Ys, op)
    alpha = ost.alpha.reshape(len(X), nrhs) @ (w * std)
    mu, _, cov, _ = O.moments_grad(O.GPState(ost.X, ost.L, alpha, op), Xq.reshape(B * q, 4), q, alpha)
    mu = mu.reshape(B, q) + float(w @ mean) + op.const_mean * (float(w @ std) - 1.0)
    Sigma = cov.reshape(B, q, q) * float((w * w * std * std).sum())
    ref = O.qlogei(mu, Sigma, O.sobol_normal_base_samples(256, q, 11), best_f)
    np.testing.assert_allclose(got, ref, rtol=1e-8, atol=1e-8)


@pytest.mark.parametrize("q", [1, 3])
def test_optimize_acqf_improves_on_raw_samples(engine, q):
    gp, X, Y, op = _model(n=300, d=3)
    best_f = float(Y.max())
    if q == 1:
        a = acqf.LogExpectedImprovement(gp, best_f=best_f)
    else:
        a = acqf.qLogExpectedImprovement(gp, best_f=best_f, sampler=acqf.SobolQMCNormalSampler(torch.Size([128]), 4))
    bounds = torch.tensor([[0.0] * 3, [1.0] * 3], dtype=torch.float64)
    X0 = acqf.gen_batch_initial_conditions(a, bounds.to(DEV), q, 4, 128, seed=5)
    with torch.no_grad():
        v0s = a(X0)
        v0 = v0s.max().item()
    Xall, vall = acqf.optimize_acqf(a, bounds, q=q, num_restarts=4, raw_samples=128,
                                    options={"batch_limit": 2, "maxiter": 50}, seed=5, return_best_only=False)
    assert bool((vall >= v0s - 1e-9).all()), (vall, v0s)
    assert vall.sum().item() > v0s.sum().item()  # L-BFGS-B made progress
    cand, val = acqf.optimize_acqf(a, bounds, q=q, num_restarts=4, raw_samples=128,
                                   options={"batch_limit": 2, "maxiter": 50}, seed=5)
    assert cand.shape == (q, 3)
    assert float(cand.min()) >= 0.0 and float(cand.max()) <= 1.0
    assert val.item() >= v0 - 1e-9
    cand2, val2 = acqf.optimize_acqf(a, bounds, q=q, num_restarts=4, raw_samples=128,
                                     options={"batch_limit": 2, "maxiter": 50}, seed=5)
    assert torch.equal(cand, cand2)
