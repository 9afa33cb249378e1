"""Independent per-output hyperparameters: the reference's multi-output SingleTaskGP on the GPU.

optimization/Bayesian1.py:108-116 fits SingleTaskGP(train_X, train_Y[n, 8], Standardize(m=8)) — a batch of 8 independent
GPs on one X, each with its own lengthscales, outputscale, noise and constant mean [upstream] — and
optimization/Bayesian6.py:474-478 keeps per-output noise and means.  The engine serves it with ONE batched call
(gpx_fit_*_batched_params_f64: X shared, Y read by column, a parameter set per problem), one batched MLL gradient
(gpx_mll_grad_batched_f64) and the multi-output objective sweep (gpx_acquire_argmax_multi_f64).

Checked against 8 separate oracle fits (one per output, its own parameters): alpha, mu / sigma^2 at the parity tolerance
(|d mu| <= 1e-9 max|mu|, |d var| <= 1e-9 k(x, x)), every output's logEI argmax and the mean-of-8 objective argmax bit for
bit (with the margin guard: the runner-up must sit below the winner by more than the score error), each output equal bit
for bit to a single fit with its parameters, and the per-output jitter retry (psd_safe_cholesky adds jitter only to the
failing batch members [upstream]).
"""
import os

import numpy as np
import pytest
import torch

from bayesianoptimizer_amd import KernelParams
from bayesianoptimizer_amd.models import ExactGP, LogExpectedImprovement
from oracle import gp_oracle as O
from tests.conftest import GOLDEN
from tests.oracle_engine import to_oracle_params
from tests.test_gpu_parity import check_argmax, check_posterior, t

pytestmark = pytest.mark.gpu


def output_params(kind, d, T, seed):
    """T distinct parameter sets: lengthscales, outputscale, noise, constant mean and linear variances all differ."""
    rng = np.random.default_rng(seed)
    ps = []
    for _ in range(T):
        ps.append(KernelParams(kind, list(0.25 + 0.6 * rng.random(d)), outputscale=0.5 + rng.random(),
                               noise=10.0 ** rng.uniform(-4, -2), const_mean=rng.uniform(-0.5, 0.5),
                               linear_variance=list(0.05 + 0.3 * rng.random(d))))
    return ps


def problem(n, d, T, seed):
    rng = np.random.default_rng(seed)
    X = rng.random((n, d))
    W = rng.standard_normal((d, T))
    Y = np.sin(3.0 * X @ W) + 0.05 * rng.standard_normal((n, T))
    return X, Y


def margin_guard(scores_ref, err, what):
    """The argmax is meaningful only if the winner beats the runner-up by more than the score error."""
    s = np.sort(scores_ref[np.isfinite(scores_ref)])[::-1]
    if s.size > 1:
        assert s[0] - s[1] > 2.0 * err, f"{what}: near-tie (gap {s[0] - s[1]:.3e} vs error {err:.3e})"


@pytest.mark.parametrize("inverse", [False, True])
@pytest.mark.parametrize("n,d,kind", [(300, 5, "scale_linear_matern52"), (1100, 8, "rbf"), (129, 3, "matern52")])
def test_fit_outputs_match_separate_oracle_fits(engine, n, d, kind, inverse):
    T = 8
    X, Y = problem(n, d, T, seed=n + d)
    ps = output_params(kind, d, T, seed=n)
    states = engine.fit_outputs(t(X), t(Y), ps, inverse=inverse)
    Xs = np.random.default_rng(5).random((1500, d))
    for q in range(T):
        op = to_oracle_params(ps[q], d)
        ost = O.fit(X, Y[:, q], op)
        a = states[q].alpha[:n, 0].cpu().numpy()
        assert np.abs(a - ost.alpha).max() <= 1e-8 * np.abs(ost.alpha).max()
        mu, var = engine.posterior(states[q], t(Xs))
        mu_r, var_r = O.posterior(ost, Xs)
        check_posterior(mu.cpu().numpy()[:, 0], var.cpu().numpy(), mu_r, var_r, O.kernel_diag(Xs, op))
        # every output's own logEI argmax
        bf = float(Y[:, q].max())
        _, bi, sc = engine.acquire(states[q], t(Xs), "logei", best_f=bf, return_scores=True)
        sref = O.acquisition(mu_r, var_r, O.ACQ_LOGEI, bf)
        check_argmax(int(bi.item()), sref, sc.cpu().numpy(), f"output {q} logEI")
        # bit for bit the single fit with this output's parameters
        single = engine.fit(t(X), t(Y[:, q:q + 1]), ps[q], inverse=inverse)
        assert torch.equal(single.alpha, states[q].alpha), f"output {q}: batched alpha differs from its single fit"
        assert torch.equal(torch.tril(single.L), torch.tril(states[q].L))


def test_exact_gp_independent_outputs_and_objective_sweeps(engine):
    """ExactGP with a parameter set per output (Standardize per column): posterior of all 8 outputs, the mean-of-8
    logEI objective (Bayesian1.py:119-140's objective, analytic form) and the variance-sum score over independent
    outputs (Bayesian7.py:671's pool-scan score) against the oracle."""
    from bayesianoptimizer_amd.transforms import Standardize

    n, d, T = 600, 5, 8
    X, Y = problem(n, d, T, seed=3)
    ps = output_params("scale_linear_matern52", d, T, seed=4)
    gp = ExactGP(X, Y, ps, outcome_transform=Standardize(), engine=engine).fit()
    assert gp.independent and gp.jitter_used == [0.0] * T
    ym, ys = Y.mean(0), Y.std(0, ddof=1)
    Ystd = (Y - ym) / ys
    osts = O.fit_outputs(X, Ystd, [to_oracle_params(p, d) for p in ps])
    Xs = np.random.default_rng(6).random((5000, d))
    post = gp.posterior(t(Xs))
    for q in range(T):
        mu_r, var_r = O.posterior(osts[q], Xs, ym[q], ys[q])
        check_posterior(post.mean[:, q].cpu().numpy(), post.variance[:, q].cpu().numpy(), mu_r, var_r,
                        O.kernel_diag(Xs, osts[q].params) * ys[q] ** 2)
    w = np.full(T, 1.0 / T)
    best_f = float((Y @ w).max())
    acq = LogExpectedImprovement(gp, best_f=best_f, weights=w)
    _, bi, sc = acq.sweep(t(Xs), return_scores=True)
    mu_o, var_o = O.objective_posterior(osts, Xs, w, ym, ys)
    sref = O.acquisition(mu_o, var_o, O.ACQ_LOGEI, best_f)
    sg = sc.cpu().numpy()
    err = np.abs(sg - sref).max()
    assert err <= 1e-9 * max(1.0, np.abs(sref).max())
    margin_guard(sref, err, "mean-of-8 logEI")
    check_argmax(int(bi.item()), sref, sg, "mean-of-8 logEI")
    # variance-sum score over the independent outputs (model space: unit weights, no untransform)
    _, bv, sv = engine.acquire_multi(gp.states, t(Xs), "variance", return_scores=True)
    _, var_sum = O.objective_posterior(osts, Xs, np.ones(T))
    assert np.abs(sv.cpu().numpy() - var_sum).max() <= 1e-9 * T
    check_argmax(int(bv.item()), var_sum, sv.cpu().numpy(), "variance sum")


def test_multi_objective_with_one_output_equals_single_sweep_bitwise(engine):
    n, d = 700, 4
    X, Y = problem(n, d, 1, seed=9)
    ps = output_params("rbf", d, 1, seed=10)
    states = engine.fit_outputs(t(X), t(Y), ps)
    Xs = t(np.random.default_rng(11).random((70000, d)))
    for kind in ("ei", "logei", "ucb", "variance"):
        v1, i1, s1 = engine.acquire(states[0], Xs, kind, best_f=0.3, beta=2.0, y_mean=0.2, y_scale=1.7,
                                    return_scores=True)
        v2, i2, s2 = engine.acquire_multi(states, Xs, kind, best_f=0.3, beta=2.0, weights=[1.0], y_mean=[0.2],
                                          y_scale=[1.7], return_scores=True)
        assert torch.equal(s1, s2), kind
        assert int(i1.item()) == int(i2.item()) and float(v1.item()) == float(v2.item())


def test_fit_outputs_per_output_jitter_retry(engine):
    """One output at noise 0 on duplicated rows fails at jitter 0 and takes the next jitter of the schedule; the others
    keep jitter 0 — each output settles where its own oracle fit does, with the same failed pivot."""
    from bayesianoptimizer_amd.models import reference_jitter_schedule

    n, d, T = 400, 3, 4
    X, Y = problem(n, d, T, seed=12)
    X[200:210] = X[100:110]  # duplicate rows: singular without noise
    ps = output_params("matern52", d, T, seed=13)
    ps[2] = ps[2].replace(noise=0.0)
    gp = ExactGP(X, Y, ps, engine=engine).fit()
    want = []
    for q in range(T):
        ost, jit, failed = O.fit_with_jitter(X, Y[:, q], to_oracle_params(ps[q], d), list(reference_jitter_schedule()))
        want.append((jit, failed))
        assert np.abs(gp.states[q].alpha[:n, 0].cpu().numpy() - ost.alpha).max() <= 1e-7 * np.abs(ost.alpha).max()
    assert gp.jitter_used == [w[0] for w in want]
    assert gp.jitter_used[2] > 0.0 and gp.jitter_used[0] == 0.0
    # the duplicated block makes K exactly singular: the Schur complements of rows 200-209 are rounding-level, so which
    # of them turns non-positive first is not defined by the arithmetic — both sides must fail inside the block, on
    # the same attempts (the real-data test pins an exact pivot where it is well determined, tests/test_gpu_realdata.py)
    assert [q for (q, _, _) in gp.pivot_failures] == [2] * len(want[2][1])
    assert all(200 <= p < 210 for (_, _, p) in gp.pivot_failures) and all(200 <= p < 210 for p in want[2][1])


def test_mll_grad_outputs_match_oracle(engine):
    n, d, T = 257, 4, 5
    X, Y = problem(n, d, T, seed=14)
    ps = output_params("scale_linear_matern52", d, T, seed=15)
    res, _ = engine.mll_value_grad_outputs(t(X), t(Y), ps)
    for q in range(T):
        ref = O.mll_value_grad(X, Y[:, q], to_oracle_params(ps[q], d))
        g = res[q]
        assert abs(g["nll"] - ref["nll"]) <= 1e-9 * abs(ref["nll"])
        for key in ("noise", "outputscale", "const_mean"):
            assert abs(g[key] - ref[key]) <= 1e-8 * max(1.0, abs(ref[key])), (q, key)
        for key in ("lengthscale", "linear_variance"):
            assert np.abs(g[key] - ref[key]).max() <= 1e-8 * max(1.0, np.abs(ref[key]).max()), (q, key)


def test_fit_hyperparameters_independent_outputs_gpu_matches_oracle_objective(engine):
    """One L-BFGS-B over the concatenated per-output vector (the sum of the per-output losses).  Parity: the summed
    objective and its gradient on the GPU equal the oracle's at equal parameters (1e-11 / 1e-9).  The optimisation: both
    runs reach the same optimum — loss within 1e-4 relative and every output's lengthscales within 2e-2, a sanity bound,
    not a parity claim (as in tests/test_mll.py: once two L-BFGS-B paths differ by rounding, scipy's relative-reduction
    stop fires at different iterates of a flat optimum) — and the outputs get parameters of their own."""
    from bayesianoptimizer_amd.mll import default_spec, fit_hyperparameters_outputs, objective_outputs

    n, d, T = 120, 3, 3
    rng = np.random.default_rng(16)
    X = rng.random((n, d))
    Y = np.stack([np.sin((4 + 2 * q) * X + q).sum(1) for q in range(T)], 1) + 0.05 * rng.standard_normal((n, T))

    def oracle_all(pl):
        return [O.mll_value_grad(X, Y[:, q], to_oracle_params(p, d)) for q, p in enumerate(pl)]

    specs = [default_spec("rbf", d, "dim_scaled", None, True) for _ in range(T)]
    raw0 = np.concatenate([sp.x0() for sp in specs])
    state = [None]

    def gpu_all(pl):
        res, state[0] = engine.mll_value_grad_outputs(t(X), t(Y), pl, states=state[0])
        return res

    # the start and a multiplicative perturbation of it (stays inside the positive domains; the means move off 0)
    raw1 = raw0 * (1.0 + 0.1 * np.random.default_rng(18).standard_normal(raw0.size)) + \
        0.05 * np.concatenate([[h.name == "const_mean" for h in sp.hypers] for sp in specs])
    for raw in (raw0, raw1):
        fg, gg = objective_outputs(specs, gpu_all, n)(raw)
        fr, gr = objective_outputs(specs, oracle_all, n)(raw)
        assert np.isfinite(fr)
        assert abs(fg - fr) <= 1e-11 * max(1.0, abs(fr)) and np.abs(gg - gr).max() <= 1e-9 * max(1.0, np.abs(gr).max())
    gpu = fit_hyperparameters_outputs(engine, t(X), t(Y), "rbf", "dim_scaled")  # scipy's L-BFGS-B defaults
    ref = fit_hyperparameters_outputs(None, X, Y, "rbf", "dim_scaled", value_grad_all=oracle_all)
    assert len(gpu.params) == T and gpu.success
    assert abs(gpu.loss - ref.loss) <= 1e-4 * max(1.0, abs(ref.loss)), (gpu.loss, ref.loss)
    for pg, pr in zip(gpu.params, ref.params):
        assert np.allclose(pg.lengthscales(d), pr.lengthscales(d), rtol=2e-2)
    ls = np.array([p.lengthscales(d) for p in gpu.params])
    assert np.ptp(ls[:, 0]) > 0.05  # the outputs got their own lengthscales


def test_reference_results_r3000_eight_outputs_own_parameters(engine):
    """The reference's own 3000-row results file, 8 outputs with 8 different parameter sets (Bayesian6's covariance,
    per-output noise / mean / scales), in one batched call, against 8 oracle fits on 2048 validation rows."""
    z = np.load(os.path.join(GOLDEN, "results_r3000.npz"))
    X, Yraw = z["X"], z["Y"]
    bounds = np.array([(0.3, 1.0), (0.001, 300.0), (0.001, 400.0), (2.0, 7.0), (2.0, 7.0)])
    Xu = (X - bounds[:, 0]) / (bounds[:, 1] - bounds[:, 0])
    Yl = np.log(Yraw - min(Yraw.min(), 0.0) + 1e-6)
    Y = (Yl - Yl.mean(0)) / Yl.std(0, ddof=1)
    Xv = (np.load(os.path.join(GOLDEN, "validation_2048.npz"))["X"] - bounds[:, 0]) / (bounds[:, 1] - bounds[:, 0])
    n, d = Xu.shape
    T = Y.shape[1]
    ps = output_params("scale_linear_matern52", d, T, seed=17)
    ps = [p.replace(noise=max(p.noise, 1e-4)) for p in ps]
    gp = ExactGP(Xu, Y, ps, engine=engine).fit()
    post = gp.posterior(t(Xv))
    osts = []
    for q in range(T):
        ost, jit, _ = O.fit_with_jitter(Xu, Y[:, q], to_oracle_params(ps[q], d))
        assert gp.jitter_used[q] == jit
        osts.append(ost)
        mu_r, var_r = O.posterior(ost, Xv)
        check_posterior(post.mean[:, q].cpu().numpy(), post.variance[:, q].cpu().numpy(), mu_r, var_r,
                        O.kernel_diag(Xv, ost.params))
        bf = float(Y[:, q].max())
        _, bi, sc = LogExpectedImprovement(gp, best_f=bf, output=q).sweep(t(Xv), return_scores=True)
        check_argmax(int(bi.item()), O.acquisition(mu_r, var_r, O.ACQ_LOGEI, bf), sc.cpu().numpy(), f"r3000 out {q}")
    w = np.full(T, 1.0 / T)
    bf = float((Y @ w).max())
    _, bi, sc = LogExpectedImprovement(gp, best_f=bf, weights=w).sweep(t(Xv), return_scores=True)
    mu_o, var_o = O.objective_posterior(osts, Xv, w)
    sref = O.acquisition(mu_o, var_o, O.ACQ_LOGEI, bf)
    err = np.abs(sc.cpu().numpy() - sref).max()
    margin_guard(sref, err, "r3000 mean-of-8 logEI")
    check_argmax(int(bi.item()), sref, sc.cpu().numpy(), "r3000 mean-of-8 logEI")


def test_per_output_entry_points_reject_invalid_arguments(engine):
    """The C ABI's validation of the round-6 entry points: a bad parameter set names its problem, mixed input dimensions,
    negative read-only strides and overlapping outputs, and a multi-output sweep over outputs of different n."""
    import ctypes

    from bayesianoptimizer_amd import GPXError
    from bayesianoptimizer_amd._capi import KernelParamsC

    n, d, T = 200, 3, 3
    X, Y = problem(n, d, T, seed=19)
    ps = output_params("rbf", d, T, seed=20)
    with pytest.raises(GPXError, match="problem 1"):
        engine.fit_outputs(t(X), t(Y), [ps[0], ps[1].replace(lengthscale=[0.3, -1.0, 0.2]), ps[2]])
    with pytest.raises(ValueError):
        engine.fit_outputs(t(X), t(Y), ps[:2])  # one parameter set per output
    states = engine.fit_outputs(t(X), t(Y), ps)
    lib, h = engine.lib, engine.handle
    pcs = (KernelParamsC * T)(*[p.to_c(d) for p in ps])
    pcs[2].d = 2  # mixed input dimensions
    Lb, Wb, Db, Ab, Ib = states[0]._batch
    nbytes = ctypes.c_size_t()
    lib.gpx_fit_factor_batched_workspace_size(n, 1, T, ctypes.byref(nbytes))
    ws = torch.empty(nbytes.value, dtype=torch.uint8, device=engine.device)
    Xt, Yt = t(X), t(Y)
    p_ = lambda v: ctypes.c_void_p(v.data_ptr())  # noqa: E731
    npad = Lb.shape[1]

    def call(pc, sx, sy, sk):
        return lib.gpx_fit_factor_batched_params_f64(h, pc, T, n, p_(Xt), d, sx, p_(Yt), T, sy, 1, p_(Lb), npad, sk,
                                                     p_(Db), Db.stride(0), p_(Ab), Ab.stride(0), p_(Ib), p_(ws),
                                                     ws.numel())

    assert call(pcs, 0, 1, Lb.stride(0)) != 0
    assert "same input dimension" in lib.gpx_last_error(h).decode()
    pcs[2].d = d
    assert call(pcs, -1, 1, Lb.stride(0)) != 0      # negative read-only stride
    assert call(pcs, 0, 1, 0) != 0                  # overlapping factors
    assert call(pcs, 0, 1, Lb.stride(0)) == 0       # and the valid call goes through
    X2, Y2 = problem(n + 5, d, 1, seed=21)
    other = engine.fit_outputs(t(X2), t(Y2), ps[:1])
    with pytest.raises(ValueError):
        engine.acquire_multi([states[0], other[0]], t(np.random.default_rng(1).random((64, d))), "logei")
