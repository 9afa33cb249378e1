"""GPU parity of the incremental posterior update (gpx_append_f64).

The bordered Cholesky of the appended rows must give the posterior a fresh fit of all rows gives (same 1e-9 relative
scale as tests/test_gpu_parity.py) and the oracle's refit; the factor itself is compared on its lower triangle.
"""
import numpy as np
import pytest
import torch

from bayesianoptimizer_amd import NotPositiveDefiniteError
from oracle import gp_oracle as O
from tests.test_gpu_parity import DEV, check_argmax, check_posterior, pair, t

pytestmark = pytest.mark.gpu


def _problem(n, d, nrhs, seed):
    X, y = O.synthetic_problem(n, d, seed)
    Y = np.stack([y * (r + 1) - r for r in range(nrhs)], axis=1)
    return X, Y


def _compare_states(engine, st, ref, n, atol_scale=1e-9):
    engine.inverse(st)
    engine.inverse(ref)
    Lg = torch.tril(st.L[:n, :n]).cpu().numpy()
    Lr = torch.tril(ref.L[:n, :n]).cpu().numpy()
    assert np.abs(Lg - Lr).max() <= atol_scale * np.abs(Lr).max()
    Wg = torch.triu(st.W[:n, :n]).cpu().numpy()
    Wr = torch.triu(ref.W[:n, :n]).cpu().numpy()
    assert np.abs(Wg - Wr).max() <= 1e-8 * np.abs(Wr).max()
    # padded rows / columns beyond n: identity factor, zero alpha
    npad = st.npad
    if npad > n:
        assert torch.equal(st.alpha[n:], torch.zeros_like(st.alpha[n:]))
        np.testing.assert_array_equal(torch.tril(st.L[n:npad, n:npad]).cpu().numpy(), np.eye(npad - n))


@pytest.mark.parametrize("kind", ["rbf", "matern52", "scale_linear_matern52"])
@pytest.mark.parametrize("n_old,q", [(100, 5), (256, 1), (300, 64), (1000, 200), (1024, 130), (2000, 700)])
def test_append_matches_refit_and_oracle(engine, kind, n_old, q):
    d, nrhs = 6, 2
    n = n_old + q
    X, Y = _problem(n, d, nrhs, n_old + 7 * q)
    kp, op = pair(kind, d, noise=2e-4, outputscale=1.3)
    st = engine.fit(t(X[:n_old]), t(Y[:n_old]), kp, capacity=n)
    ld0 = st.L.stride(0)
    st = engine.append(st, t(X), t(Y))
    assert st.n == n and st.L.stride(0) == ld0  # grew in place
    ref = engine.fit(t(X), t(Y), kp)
    _compare_states(engine, st, ref, n)
    a_ref = ref.alpha[:n].cpu().numpy()
    assert np.abs(st.alpha[:n].cpu().numpy() - a_ref).max() <= 1e-8 * np.abs(a_ref).max()
    ost = O.fit(X, Y, op)
    Xq = O.sobol_candidates(512, d, 3)
    mu, var = engine.posterior(st, t(Xq))
    mu_r, var_r = O.posterior(ost, Xq)
    check_posterior(mu.cpu().numpy(), var.cpu().numpy(), mu_r, var_r, O.kernel_diag(Xq, op))
    bv, bi, sg = engine.acquire(st, t(Xq), "logei", best_f=float(Y[:, 0].max()), return_scores=True)
    sref = O.acquisition(*O.posterior(O.GPState(X, ost.L, ost.alpha[:, 0], op), Xq), O.ACQ_LOGEI,
                         best_f=float(Y[:, 0].max()))
    check_argmax(int(bi.item()), sref, sg.cpu().numpy(), f"append {kind}")


def test_append_sequence_grows_buffers(engine):
    # several appends of a few points each, starting without spare capacity (buffers are regrown on the way)
    d = 5
    X, Y = _problem(900, d, 1, 11)
    kp, op = pair("matern52", d, noise=1e-4)
    st = engine.fit(t(X[:150]), t(Y[:150]), kp)
    for n in (151, 170, 256, 257, 400, 640, 900):
        st = engine.append(st, t(X[:n]), t(Y[:n]))
    ref = engine.fit(t(X), t(Y), kp)
    _compare_states(engine, st, ref, 900)
    ost = O.fit(X, Y, op)
    Xq = O.sobol_candidates(300, d, 5)
    mu, var = engine.posterior(st, t(Xq))
    mu_r, var_r = O.posterior(ost, Xq)
    check_posterior(mu.cpu().numpy(), var.cpu().numpy(), mu_r, var_r, O.kernel_diag(Xq, op))


def test_append_restandardised_targets(engine):
    # the reference re-standardises Y every round: only alpha changes, the factor is kept
    from bayesianoptimizer_amd.transforms import Standardize

    d = 4
    X, Y = _problem(500, d, 3, 21)
    kp, op = pair("rbf", d, noise=1e-3)
    Ys_old = Standardize().fit(t(Y[:400])).transform(t(Y[:400]))
    st = engine.fit(t(X[:400]), Ys_old, kp, capacity=500)
    Ys = Standardize().fit(t(Y)).transform(t(Y))
    st = engine.append(st, t(X), Ys)
    ost = O.fit(X, Ys.cpu().numpy(), op)
    a_r = ost.alpha
    assert np.abs(st.alpha[:500].cpu().numpy() - a_r).max() <= 1e-7 * np.abs(a_r).max()


def test_append_not_pd_reports_global_pivot(engine):
    d = 3
    X, _ = O.synthetic_problem(256, d, 1)
    # two appended copies of a point far from all others: K21 = 0 exactly, and with no noise the second copy's
    # pivot is 1 - 1*1 = 0 exactly (global index 257)
    X = np.vstack([X, [[50.0] * d], [[50.0] * d], [[0.5] * d]])
    kp, _ = pair("rbf", d, ls=0.05, noise=0.0)  # short lengthscale: the old Gram is well conditioned without noise
    st = engine.fit(t(X[:256]), t(np.zeros(256)), kp, capacity=300)
    with pytest.raises(NotPositiveDefiniteError) as e:
        engine.append(st, t(X), t(np.zeros(259)))
    assert e.value.pivot == 257


def test_append_invalid_arguments(engine):
    d = 3
    X, Y = _problem(200, d, 1, 2)
    kp, _ = pair("rbf", d)
    st = engine.fit(t(X[:100]), t(Y[:100]), kp)
    with pytest.raises(ValueError):
        engine.append(st, t(X[:100]), t(Y[:100]))  # nothing new
    with pytest.raises(ValueError):
        engine.append(st, t(X[:, :2]), t(Y))  # wrong d


def test_exact_gp_append_observations_matches_refit(engine):
    from bayesianoptimizer_amd.models import ExactGP
    from bayesianoptimizer_amd.transforms import Standardize

    d = 5
    X, Y = _problem(700, d, 2, 31)
    kp, _ = pair("rbf", d, noise=1e-3)
    gp = ExactGP(X[:500], Y[:500], kp, outcome_transform=Standardize(), engine=engine).fit()
    gp.append_observations(X[500:600], Y[500:600])
    gp.append_observations(X[600:], Y[600:])
    ref = ExactGP(X, Y, kp, outcome_transform=Standardize(), engine=engine).fit()
    Xq = t(O.sobol_candidates(256, d, 9))
    pa, pr = gp.posterior(Xq), ref.posterior(Xq)
    assert gp.state.n == 700
    assert (pa.mean - pr.mean).abs().max().item() <= 1e-9 * pr.mean.abs().max().item()
    assert (pa.variance - pr.variance).abs().max().item() <= 1e-9 * pr.variance.abs().max().item()
