"""Marginal-likelihood hyperparameter fit.

CPU: the oracle's -log p(y) gradient against central finite differences (pins the derivative formulas), the
host-side objective (priors, transforms, 1/n scaling) against finite differences of itself, and the L-BFGS-B
driver on the oracle.  GPU: gpx_mll_grad_f64 against the oracle, and the whole GPU-driven fit against the
oracle-driven fit.

Tolerances: value |d nll| <= 1e-10 * (|quad| + |logdet| + n); gradient |d g| <= 1e-8 * (1 + max|g|) (the
gradient contracts K^{-1} = W W^T, whose rounding grows with cond(K); the tests use noise >= 1e-3).
Parity unpinned at the BoTorch level (no gpytorch/botorch here): the prior sets restate the SingleTaskGP
defaults documented in bayesianoptimizer_amd/mll.py.
"""
import math

import numpy as np
import pytest
import torch

from bayesianoptimizer_amd import KernelParams
from bayesianoptimizer_amd.mll import default_spec, fit_hyperparameters, objective
from oracle import gp_oracle as O

KINDS = {"rbf": O.RBF, "matern52": O.MATERN52, "scale_linear_matern52": O.SCALE_LINEAR_MATERN52}


def to_oracle(p: KernelParams, d: int) -> O.KernelParams:
    return O.KernelParams(p.kind_id, np.array(p.lengthscales(d)), outputscale=p.outputscale, noise=p.noise,
                          const_mean=p.const_mean, linear_variance=np.array(p.linear_variances(d)),
                          jitter=p.jitter)


def oracle_value_grad(X, y):
    d = X.shape[1]
    return lambda p: O.mll_value_grad(X, y, to_oracle(p, d))


def problem(n, d, seed):
    X, y = O.synthetic_problem(n, d, seed)
    return X, y


# ---- CPU: oracle and host logic ------------------------------------------------------------------
@pytest.mark.parametrize("kind", list(KINDS))
def test_oracle_gradient_matches_finite_differences(kind):
    rng = np.random.default_rng(3)
    X = rng.random((50, 3))
    y = np.sin(5 * X).sum(1)
    p = O.KernelParams(KINDS[kind], [0.3, 0.5, 0.7], outputscale=1.3, noise=1e-2, const_mean=0.1,
                       linear_variance=[0.2, 0.4, 0.6])
    g = O.mll_value_grad(X, y, p)

    def f(**kw):
        dd = dict(p.__dict__)
        dd.update(kw)
        return O.mll_value_grad(X, y, O.KernelParams(**dd))["nll"]

    h = 1e-6
    for name, base in [("noise", p.noise), ("outputscale", p.outputscale), ("const_mean", p.const_mean)]:
        fd = (f(**{name: base + h}) - f(**{name: base - h})) / (2 * h)
        assert abs(fd - g[name]) <= 1e-5 * (1 + abs(fd)), (name, fd, g[name])
    for k in range(3):
        for name in ["lengthscale"] + (["linear_variance"] if kind == "scale_linear_matern52" else []):
            vp = getattr(p, name).copy()
            vm = vp.copy()
            vp[k] += h
            vm[k] -= h
            fd = (f(**{name: vp}) - f(**{name: vm})) / (2 * h)
            assert abs(fd - g[name][k]) <= 1e-5 * (1 + abs(fd)), (name, k, fd, g[name][k])


def test_oracle_nll_closed_form():
    # one point: K = s + noise, -log p = y^2 / (2K) + log(K)/2 + log(2 pi)/2
    p = O.KernelParams(O.RBF, [0.5], outputscale=2.0, noise=0.5)
    g = O.mll_value_grad(np.array([[0.3]]), np.array([1.5]), p)
    K = 2.5
    assert math.isclose(g["nll"], 1.5 ** 2 / (2 * K) + 0.5 * math.log(K) + 0.5 * math.log(2 * math.pi), rel_tol=1e-14)
    assert math.isclose(g["noise"], 0.5 / K - 1.5 ** 2 / (2 * K * K), rel_tol=1e-12)


@pytest.mark.parametrize("prior_set,kind", [("dim_scaled", "rbf"), ("dim_scaled", "matern52"), ("gamma", "matern52"),
                                            ("none", "scale_linear_matern52")])
def test_objective_chain_rule(prior_set, kind):
    X, y = problem(40, 3, 7)
    spec = default_spec(kind, 3, prior_set)
    f = objective(spec, oracle_value_grad(X, y), X.shape[0])
    rng = np.random.default_rng(0)
    raw = spec.x0() + 0.1 * rng.standard_normal(len(spec.hypers))
    for i, b in enumerate(spec.bounds()):  # stay inside the bounds for the identity-transformed entries
        if b[0] is not None:
            raw[i] = max(raw[i], b[0] * 1.5)
    v, g = f(raw)
    h = 1e-6
    for i in range(len(raw)):
        e = np.zeros_like(raw)
        e[i] = h * max(1.0, abs(raw[i]))
        fd = (f(raw + e)[0] - f(raw - e)[0]) / (2 * e[i])
        assert abs(fd - g[i]) <= 1e-5 * (1 + abs(fd)), (spec.hypers[i].name, fd, g[i])


def test_dim_scaled_defaults_match_botorch_modes():
    spec = default_spec("rbf", 8, "dim_scaled")
    p = spec.params_from_raw(spec.x0())
    assert np.allclose(p.lengthscales(8), math.exp(SQRT2_PLUS_HALF_LOG(8) - 3.0))
    assert math.isclose(p.noise, math.exp(-5.0))
    assert p.outputscale == 1.0
    names = [h.name for h in spec.hypers]
    assert names == ["noise", "const_mean"] + ["lengthscale"] * 8
    assert spec.bounds()[0] == (1e-4, None) and spec.bounds()[2] == (2.5e-2, None)


def SQRT2_PLUS_HALF_LOG(d):
    return math.sqrt(2.0) + 0.5 * math.log(d)


def test_fit_hyperparameters_oracle_reaches_stationary_point():
    X, y = problem(60, 2, 11)
    vg = oracle_value_grad(X, y)
    spec = default_spec("rbf", 2, "dim_scaled")
    f = objective(spec, vg, 60)
    v0, _ = f(spec.x0())
    res = fit_hyperparameters(None, X, y, "rbf", "dim_scaled", value_grad=vg)  # scipy defaults
    assert res.success and res.loss < v0
    # run to the precision limit: the projected gradient vanishes at the optimum
    tight = fit_hyperparameters(None, X, y, "rbf", "dim_scaled", value_grad=vg,
                                options={"ftol": 1e-15, "gtol": 1e-10, "maxiter": 2000})
    v, g = f(tight.raw)
    assert v <= res.loss + 1e-12
    for (lo, _), r, gi in zip(spec.bounds(), tight.raw, g):
        if lo is not None and r - lo < 1e-9 * max(1.0, abs(lo)):
            assert gi >= -1e-7
        else:
            assert abs(gi) < 1e-6, g


# ---- GPU: kernel parity and the GPU-driven fit ---------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("kind", list(KINDS))
@pytest.mark.parametrize("n,d", [(1, 1), (100, 3), (257, 8), (700, 5), (300, 20)])
def test_mll_grad_gpu_vs_oracle(engine, kind, n, d):
    X, y = problem(n, d, 100 + n + d)
    rng = np.random.default_rng(n)
    p = KernelParams(kind, list(0.3 + 0.6 * rng.random(d)), outputscale=1.4, noise=2e-3, const_mean=0.05,
                     linear_variance=list(0.1 + 0.5 * rng.random(d)))
    dev = engine.device
    res, _ = engine.mll_value_grad(torch.tensor(X, device=dev), torch.tensor(y, device=dev), p, jitters=(0.0,))
    ref = O.mll_value_grad(X, y, to_oracle(p, d))
    scale_v = abs(ref["quad"]) + abs(ref["logdet"]) + n
    assert abs(res["nll"] - ref["nll"]) <= 1e-10 * scale_v
    assert abs(res["logdet"] - ref["logdet"]) <= 1e-10 * scale_v
    grads = [("noise", res["noise"], ref["noise"]), ("outputscale", res["outputscale"], ref["outputscale"]),
             ("const_mean", res["const_mean"], ref["const_mean"])]
    grads += [(f"l{k}", res["lengthscale"][k], ref["lengthscale"][k]) for k in range(d)]
    grads += [(f"v{k}", res["linear_variance"][k], ref["linear_variance"][k]) for k in range(d)]
    gmax = max(abs(r) for _, _, r in grads)
    for name, a, b in grads:
        assert abs(a - b) <= 1e-8 * (1 + gmax), (name, a, b)


@pytest.mark.gpu
def test_mll_grad_gpu_deterministic(engine):
    X, y = problem(1000, 6, 5)
    p = KernelParams("matern52", 0.4, noise=1e-3)
    dev = engine.device
    Xt, yt = torch.tensor(X, device=dev), torch.tensor(y, device=dev)
    a, st = engine.mll_value_grad(Xt, yt, p)
    v1 = engine.mll_grad(st, yt).cpu().numpy()
    v2 = engine.mll_grad(st, yt).cpu().numpy()
    assert np.array_equal(v1, v2)


@pytest.mark.gpu
@pytest.mark.parametrize("prior_set,kind", [("dim_scaled", "rbf"), ("gamma", "matern52")])
def test_fit_hyperparameters_gpu_matches_oracle_driven_fit(engine, prior_set, kind):
    X, y = problem(300, 4, 21)
    gpu = fit_hyperparameters(engine, torch.tensor(X, device=engine.device), y, kind, prior_set)
    ref = fit_hyperparameters(None, X, y, kind, prior_set, value_grad=oracle_value_grad(X, y))
    assert gpu.success and ref.success
    assert abs(gpu.loss - ref.loss) <= 1e-6 * (1 + abs(ref.loss))  # default ftol: both stop near the optimum
    tight = {"ftol": 1e-15, "gtol": 1e-10, "maxiter": 2000}
    gpu = fit_hyperparameters(engine, torch.tensor(X, device=engine.device), y, kind, prior_set, options=tight)
    ref = fit_hyperparameters(None, X, y, kind, prior_set, value_grad=oracle_value_grad(X, y), options=tight)
    assert abs(gpu.loss - ref.loss) <= 1e-9 * (1 + abs(ref.loss))
    assert np.allclose(gpu.params.lengthscales(4), ref.params.lengthscales(4), rtol=1e-4)
    assert math.isclose(gpu.params.noise, ref.params.noise, rel_tol=1e-3, abs_tol=1e-7)


@pytest.mark.gpu
def test_mll_grad_full_size_finite_difference(engine):
    """n=4096 d=8 (BASELINE configs[1] shape): the GPU gradient against central differences of the GPU nll."""
    X, y = problem(4096, 8, 0)
    dev = engine.device
    Xt, yt = torch.tensor(X, device=dev), torch.tensor(y, device=dev)
    ls = np.full(8, 0.6)
    p = KernelParams("rbf", list(ls), noise=1e-2)
    g, _ = engine.mll_value_grad(Xt, yt, p)
    for k in (0, 5):
        h = 1e-5
        lp, lm = ls.copy(), ls.copy()
        lp[k] += h
        lm[k] -= h
        fp, _ = engine.mll_value_grad(Xt, yt, p.replace(lengthscale=list(lp)))
        fm, _ = engine.mll_value_grad(Xt, yt, p.replace(lengthscale=list(lm)))
        fd = (fp["nll"] - fm["nll"]) / (2 * h)
        assert abs(fd - g["lengthscale"][k]) <= 1e-4 * (1 + abs(fd)), (k, fd, g["lengthscale"][k])
    h = 1e-7
    fp, _ = engine.mll_value_grad(Xt, yt, p.replace(noise=1e-2 + h))
    fm, _ = engine.mll_value_grad(Xt, yt, p.replace(noise=1e-2 - h))
    fd = (fp["nll"] - fm["nll"]) / (2 * h)
    assert abs(fd - g["noise"]) <= 1e-4 * (1 + abs(fd))


def test_oracle_multi_output_gradient_matches_finite_differences():
    rng = np.random.default_rng(4)
    X = rng.random((30, 2))
    Y = np.stack([np.sin(4 * X).sum(1), np.cos(3 * X[:, 0]), X[:, 1] ** 2], 1)
    p = O.KernelParams(O.MATERN52, [0.4, 0.6], outputscale=0.9, noise=2e-2, const_mean=0.05)
    g = O.mll_value_grad(X, Y, p)
    single = sum(O.mll_value_grad(X, Y[:, t], p)["nll"] for t in range(3))
    assert math.isclose(g["nll"], single, rel_tol=1e-12)  # shared hyperparameters: the outputs' nll add up
    h = 1e-6
    for k in range(2):
        lp, lm = p.lengthscale.copy(), p.lengthscale.copy()
        lp[k] += h
        lm[k] -= h
        fd = (O.mll_value_grad(X, Y, O.KernelParams(O.MATERN52, lp, 0.9, 2e-2, 0.05))["nll"] -
              O.mll_value_grad(X, Y, O.KernelParams(O.MATERN52, lm, 0.9, 2e-2, 0.05))["nll"]) / (2 * h)
        assert abs(fd - g["lengthscale"][k]) <= 1e-5 * (1 + abs(fd))


def test_exact_gp_fit_hyperparameters_with_oracle_engine():
    from bayesianoptimizer_amd.models import ExactGP
    from bayesianoptimizer_amd.transforms import Standardize
    from tests.oracle_engine import OracleEngine

    X, y = problem(40, 3, 9)
    gp = ExactGP(torch.tensor(X), torch.tensor(np.stack([y, -y], 1)), KernelParams("rbf", 0.5),
                 engine=OracleEngine(), outcome_transform=Standardize())
    gp.fit_hyperparameters("dim_scaled")
    assert gp.mll_result.success and gp.state is not None
    assert gp.params.noise >= 1e-4 and min(gp.params.lengthscales(3)) >= 2.5e-2


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["rbf", "scale_linear_matern52"])
def test_mll_grad_gpu_multi_output(engine, kind):
    n, d, T = 333, 4, 5
    X, y = problem(n, d, 77)
    rng = np.random.default_rng(1)
    Y = np.stack([y * (t + 1) + 0.1 * rng.standard_normal(n) for t in range(T)], 1)
    p = KernelParams(kind, [0.5, 0.7, 0.4, 0.9], outputscale=1.2, noise=5e-3, const_mean=-0.1, linear_variance=0.3)
    dev = engine.device
    res, _ = engine.mll_value_grad(torch.tensor(X, device=dev), torch.tensor(Y, device=dev), p, jitters=(0.0,))
    ref = O.mll_value_grad(X, Y, to_oracle(p, d))
    assert abs(res["nll"] - ref["nll"]) <= 1e-10 * (abs(ref["quad"]) + T * (abs(ref["logdet"]) + n))
    names = ["noise", "outputscale", "const_mean"]
    gmax = max([abs(ref[k]) for k in names] + list(np.abs(ref["lengthscale"])))
    for k in names:
        assert abs(res[k] - ref[k]) <= 1e-8 * (1 + gmax), k
    assert np.abs(res["lengthscale"] - ref["lengthscale"]).max() <= 1e-8 * (1 + gmax)
    assert np.abs(res["linear_variance"] - ref["linear_variance"]).max() <= 1e-8 * (1 + gmax)


@pytest.mark.gpu
def test_exact_gp_fit_hyperparameters_gpu_matches_oracle_engine(engine):
    from bayesianoptimizer_amd.models import ExactGP
    from bayesianoptimizer_amd.transforms import Standardize
    from tests.oracle_engine import OracleEngine

    X, y = problem(200, 3, 12)
    Y = np.stack([y, np.cos(3 * X[:, 0])], 1)
    # run both to the precision limit: with scipy's default ftol the two L-BFGS-B paths stop at different points
    # of a flat optimum after rounding-level differences in the objective
    tight = {"ftol": 1e-15, "gtol": 1e-10, "maxiter": 2000}
    g1 = ExactGP(torch.tensor(X), torch.tensor(Y), KernelParams("matern52", 0.5), engine=engine,
                 outcome_transform=Standardize()).fit_hyperparameters("gamma", options=tight)
    g2 = ExactGP(torch.tensor(X), torch.tensor(Y), KernelParams("matern52", 0.5), engine=OracleEngine(),
                 outcome_transform=Standardize()).fit_hyperparameters("gamma", options=tight)
    # Same optimum, not the same path: the objective and gradient agree to ~1e-12 at equal parameters (the tests
    # above), but in this flat optimum L-BFGS-B's relative-reduction stop fires at different iterates once the two
    # paths differ by rounding (observed: 346 vs 408 evaluations, final losses 1e-7 apart on the same engine build
    # pair), so the end-to-end check is on the optimum's value and location.  The location is loose: along the flat
    # direction the two stops were measured 2.9e-3 apart in the lengthscales (round 3) with losses equal to 1e-6.
    assert abs(g1.mll_result.loss - g2.mll_result.loss) <= 1e-6 * (1 + abs(g2.mll_result.loss))
    assert np.allclose(g1.params.lengthscales(3), g2.params.lengthscales(3), rtol=1e-2)
