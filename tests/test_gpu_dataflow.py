"""The persistent dataflow Cholesky (gpx_potrf_dag.hip, opt-in: potrf_schedule = 2; measured slower than the default
multi-launch schedule) against the multi-launch schedule and the oracle; failure reporting of the two persistent launches (dataflow Cholesky, triangular solve) when an
in-launch hand-off times out; the per-handle options that replaced the library's environment knobs (include/gpx.h
GPX_OPT_*).  Reference call sites: psd_safe_cholesky [upstream] reached from optimization/Bayesian.py:89-94, jitter
retry optimization/Bayesian6.py:481-488."""
import os

import numpy as np
import pytest
import torch

from bayesianoptimizer_amd import GPEngine, GPXError, GPXTimeoutError, KernelParams, NotPositiveDefiniteError
from bayesianoptimizer_amd import _capi
from oracle import gp_oracle as O
from tests.test_gpu_parity import RTOL, pair, t

pytestmark = pytest.mark.gpu


def _factor(engine, X, kp, n, schedule):
    engine.set_option("potrf_schedule", schedule)
    try:
        K = engine.gram(t(X), kp)
        Dinv, info = engine.potrf(K, n)
        torch.cuda.synchronize()
    finally:
        engine.set_option("potrf_schedule", 0)
    return np.tril(K.cpu().numpy()), Dinv.cpu().numpy(), int(info.item())


@pytest.mark.parametrize("n,kind", [(1, "rbf"), (129, "matern52"), (256, "rbf"), (700, "scale_linear_matern52"),
                                    (2048, "rbf"), (4096, "rbf")])
def test_dataflow_factor_matches_multilaunch_and_oracle(engine, n, kind):
    d = 8
    X, _ = O.synthetic_problem(n, d, n + 11)
    kp, op = pair(kind, d, noise=1e-4)
    L2, D2, i2 = _factor(engine, X, kp, n, 2)
    L1, D1, i1 = _factor(engine, X, kp, n, 1)
    assert i1 == i2 == 0
    npad = L2.shape[0]
    scale = np.abs(L1).max()
    # two arrangements of the same fp64 arithmetic (aggregated trailing products vs one column per launch)
    assert np.abs(L2 - L1).max() <= 1e-12 * scale
    np.testing.assert_array_equal(L2[n:, n:], np.eye(npad - n))
    for b in range(npad // 64):
        blk = L2[64 * b:64 * b + 64, 64 * b:64 * b + 64]
        np.testing.assert_allclose(D2[b] @ blk, np.eye(64), atol=1e-10)
    if n <= 2048:
        Lr = O.cholesky(O.gram(X, op))
        assert np.abs(L2[:n, :n] - Lr).max() <= RTOL * np.abs(Lr).max()


def test_dataflow_not_pd_pivot_deep(engine):
    # a pivot in the middle of a 4096 factor (chain step 32): the dataflow schedule stops there and reports it like the
    # multi-launch schedule does
    n = 4096
    X, _ = O.synthetic_problem(n, 8, 5)
    kp, _ = pair("rbf", 8, noise=1e-4)
    piv = 2085
    for schedule in (1, 2):
        engine.set_option("potrf_schedule", schedule)
        try:
            K = engine.gram(t(X), kp)
            K[piv, piv] = -1.0
            _, info = engine.potrf(K, n)
            assert int(info.item()) == piv + 1, schedule
        finally:
            engine.set_option("potrf_schedule", 0)


def test_fit_timeout_raises_timeout_error_not_not_pd(engine):
    """spin_limit = 0: every in-launch wait gives up at its first unmet poll.  Under both schedules the fit raises
    GPXTimeoutError (dataflow: the pool tasks wait for the chain from the start; multi-launch: the backward solve's
    hand-offs), never NotPositiveDefiniteError (a jitter retry would not cure it), and the next call with the default
    limit is correct again."""
    n = 4096
    X, y = O.synthetic_problem(n, 8, 21)
    kp, _ = pair("rbf", 8, noise=1e-4)
    for schedule in (0, 2):
        engine.set_option("potrf_schedule", schedule)
        engine.set_option("spin_limit", 0)
        try:
            with pytest.raises(GPXTimeoutError):
                engine.fit(t(X), t(y), kp)
        finally:
            engine.set_option("spin_limit", 1 << 22)
            engine.set_option("potrf_schedule", 0)
    st = engine.fit(t(X), t(y), kp)
    assert st.pivot_failure() == -1


def test_potrs_timeout_reported_in_info(engine):
    """The triangular solve alone (multi-launch Cholesky, which never spins): a timed-out hand-off writes
    GPX_INFO_TIMEOUT into the problem's info word instead of leaving NaN scores behind silently."""
    n = 4096
    X, y = O.synthetic_problem(n, 8, 22)
    kp, _ = pair("rbf", 8, noise=1e-4)
    engine.set_option("potrf_schedule", 1)
    engine.set_option("spin_limit", 0)
    try:
        st = engine.fit(t(X), t(y), kp, check=False)
        assert int(st.info.item()) == _capi.GPX_INFO_TIMEOUT
        with pytest.raises(GPXTimeoutError):
            st.pivot_failure()
        with pytest.raises(GPXTimeoutError):
            st.check()
    finally:
        engine.set_option("spin_limit", 1 << 22)
        engine.set_option("potrf_schedule", 0)


def test_batched_timeout_names_the_problem(engine):
    n, B = 1000, 3
    X = np.stack([O.synthetic_problem(n, 5, 30 + b)[0] for b in range(B)])
    Y = np.stack([O.synthetic_problem(n, 5, 30 + b)[1] for b in range(B)])
    kp, _ = pair("rbf", 5, noise=1e-4)
    engine.set_option("spin_limit", 0)
    try:
        with pytest.raises(GPXTimeoutError, match="problem"):
            engine.fit_batched(t(X), t(Y), kp)
    finally:
        engine.set_option("spin_limit", 1 << 22)
    sts = engine.fit_batched(t(X), t(Y), kp)
    assert [s.pivot_failure() for s in sts] == [-1] * B


def test_options_roundtrip_and_validation(engine):
    for name, value in (("potrf_schedule", 2), ("spin_limit", 12345), ("sweep_fused", 0), ("gram_split", 2),
                        ("potrf_lazy", 3), ("potrf_mode", 1)):
        old = engine.get_option(name)
        engine.set_option(name, value)
        assert engine.get_option(name) == value
        engine.set_option(name, old)
        assert engine.get_option(name) == old
    for name, bad in (("potrf_schedule", 3), ("spin_limit", -1), ("sweep_fused", 2), ("gram_split", 3),
                      ("potrf_lazy", 17), ("potrf_mode", 2)):
        with pytest.raises(GPXError) as e:
            engine.set_option(name, bad)
        assert e.value.status == _capi.GPX_INVALID_ARG
    assert engine.lib.gpx_set_option(engine.handle, 99, 0) == _capi.GPX_INVALID_ARG


def test_options_from_environment_at_create():
    os.environ["GPX_OPTIONS"] = "potrf_schedule=1,sweep_fused=0,spin_limit=777,bogus=5"
    try:
        e2 = GPEngine("cuda:0")
    finally:
        del os.environ["GPX_OPTIONS"]
    assert e2.get_option("potrf_schedule") == 1
    assert e2.get_option("sweep_fused") == 0
    assert e2.get_option("spin_limit") == 777
    assert e2.get_option("gram_split") == 0


def test_fit_results_identical_across_pool_sizes(engine):
    """The dataflow schedule decides who runs a task, never how: a batched fit (64 workgroups per problem) equals the
    single fit (256 workgroups) bit for bit at n = 4096; so does the default multi-launch schedule."""
    n = 4096
    X, y = O.synthetic_problem(n, 8, 40)
    kp, _ = pair("rbf", 8, noise=1e-4)
    for schedule in (2, 0):
        engine.set_option("potrf_schedule", schedule)
        try:
            st = engine.fit(t(X), t(y), kp)
            L1 = st.L.cpu().numpy().copy()
            sts = engine.fit_batched(t(np.stack([X] * 4)), t(np.stack([y] * 4)), kp)
            for s in sts:
                np.testing.assert_array_equal(np.tril(s.L.cpu().numpy()), np.tril(L1))
        finally:
            engine.set_option("potrf_schedule", 0)


def test_matrix_leading_dimension_limit(engine):
    """Matrix leading dimensions above GPX_MAX_LD (2^20: the tile stores use buffer descriptors with 32-bit byte
    offsets) are rejected with GPX_INVALID_ARG before anything runs; the pointers are never dereferenced."""
    K = torch.zeros(128, 128, dtype=torch.float64, device=engine.device)
    Dinv = torch.zeros(4, 64, 64, dtype=torch.float64, device=engine.device)  # 2 (npad / 64) blocks
    info = torch.zeros(1, dtype=torch.int32, device=engine.device)
    p = lambda x: x.data_ptr()
    st = engine.lib.gpx_potrf_f64(engine.handle, 128, p(K), (1 << 20) + 2, p(Dinv), p(info))
    assert st == _capi.GPX_INVALID_ARG
    assert b"GPX_MAX_LD" in engine.lib.gpx_last_error(engine.handle)
    assert engine.lib.gpx_potrf_f64(engine.handle, 128, p(K), 128, p(Dinv), p(info)) == _capi.GPX_OK
    torch.cuda.synchronize()
    assert int(info.item()) != 0  # the all-zero matrix is not positive definite
