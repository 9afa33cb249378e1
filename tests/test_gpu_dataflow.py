"""Failure reporting of the persistent launches (the triangular solve's hand-offs) when an in-launch hand-off times
out, the per-handle options that replaced the library's environment knobs (include/gpx.h GPX_OPT_*), the pivot of a
failing factorisation deep in the matrix (eager and lookahead panel schedules), batch invariance of the factor, and the
leading-dimension limit.  Reference call sites: psd_safe_cholesky [upstream] reached from
optimization/Bayesian.py:89-94, jitter retry optimization/Bayesian6.py:481-488."""
import ctypes
import os

import numpy as np
import pytest
import torch

from bayesianoptimizer_amd import GPEngine, GPXError, GPXTimeoutError, KernelParams, NotPositiveDefiniteError
from bayesianoptimizer_amd import _capi
from oracle import gp_oracle as O
from tests.test_gpu_parity import RTOL, pair, t

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,piv", [
    (4096, 300),    # block column 4: the lookahead start of a single 64-block fit (launches c < 9)
    (4096, 2085),   # block column 32: the eager part after the switch, split panels
    (8320, 3000),   # 130 blocks: lookahead schedule with lazy flushes
    (8320, 7000),   # block column 109: the eager tail (last ~32 block columns)
])
def test_not_pd_pivot_deep(engine, n, piv):
    """A failing pivot deep in the matrix stops the factorisation there and is reported as info = pivot + 1 under the
    DEFAULT schedules (the hybrid lookahead -> eager single fit and the eager tail above 64 blocks) and under
    the forced eager / lookahead options."""
    X, _ = O.synthetic_problem(n, 8, 5)
    kp, _ = pair("rbf", 8, noise=1e-4)
    for mode, lazy in ((-1, 0), (0, 1), (1, 4)):
        engine.set_option("potrf_mode", mode)
        engine.set_option("potrf_lazy", lazy)
        try:
            K = engine.gram(t(X), kp)
            K[piv, piv] = -1.0
            _, info = engine.potrf(K, n)
            assert int(info.item()) == piv + 1, (mode, lazy)
        finally:
            engine.set_option("potrf_mode", -1)
            engine.set_option("potrf_lazy", 0)


def test_fit_timeout_raises_timeout_error_not_not_pd(engine):
    """spin_limit = 0: every in-launch wait gives up at its first unmet poll.  The fit raises GPXTimeoutError (the
    backward solve's hand-offs), never NotPositiveDefiniteError (a jitter retry would not cure it), and the next call
    with the default limit is correct again."""
    n = 4096
    X, y = O.synthetic_problem(n, 8, 21)
    kp, _ = pair("rbf", 8, noise=1e-4)
    engine.set_option("spin_limit", 0)
    try:
        with pytest.raises(GPXTimeoutError):
            engine.fit(t(X), t(y), kp)
    finally:
        engine.set_option("spin_limit", 1 << 22)
    st = engine.fit(t(X), t(y), kp)
    assert st.pivot_failure() == -1


def test_potrs_timeout_reported_in_info(engine):
    """The triangular solve alone (multi-launch Cholesky, which never spins): a timed-out hand-off writes
    GPX_INFO_TIMEOUT into the problem's info word instead of leaving NaN scores behind silently."""
    n = 4096
    X, y = O.synthetic_problem(n, 8, 22)
    kp, _ = pair("rbf", 8, noise=1e-4)
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
    for name, value in (("spin_limit", 12345), ("sweep_fused", 0), ("gram_split", 2),
                        ("potrf_lazy", 3), ("potrf_mode", 1), ("potrf_switch", 13)):
        old = engine.get_option(name)
        engine.set_option(name, value)
        assert engine.get_option(name) == value
        engine.set_option(name, old)
        assert engine.get_option(name) == old
    for name, bad in (("spin_limit", -1), ("sweep_fused", 2), ("gram_split", 3),
                      ("potrf_lazy", 17), ("potrf_mode", 2), ("potrf_switch", -2)):
        with pytest.raises(GPXError) as e:
            engine.set_option(name, bad)
        assert e.value.status == _capi.GPX_INVALID_ARG
    assert engine.lib.gpx_set_option(engine.handle, 99, 0) == _capi.GPX_INVALID_ARG
    assert engine.lib.gpx_set_option(engine.handle, _capi.GPX_OPT_COUNT, 0) == _capi.GPX_INVALID_ARG
    v = ctypes.c_int64()
    for slot in _capi.GPX_OPT_RESERVED:  # a removed option's number is never reused
        assert engine.lib.gpx_set_option(engine.handle, slot, 0) == _capi.GPX_INVALID_ARG
        assert engine.lib.gpx_get_option(engine.handle, slot, ctypes.byref(v)) == _capi.GPX_INVALID_ARG


def test_options_from_environment_at_create(capfd):
    os.environ["GPX_OPTIONS"] = "potrf_mode=1,sweep_fused=0,spin_limit=777,bogus=5,potrf_schedule=1,gram_split=3"
    try:
        e2 = GPEngine("cuda:0")
    finally:
        del os.environ["GPX_OPTIONS"]
    err = capfd.readouterr().err
    # unknown names and invalid values are reported, not dropped silently
    assert "unknown option 'bogus'" in err and "unknown option 'potrf_schedule'" in err and "gram_split" in err
    assert e2.get_option("potrf_mode") == 1
    assert e2.get_option("sweep_fused") == 0
    assert e2.get_option("spin_limit") == 777
    assert e2.get_option("gram_split") == 0


# (potrf_mode, potrf_lazy, potrf_switch): eager, lookahead with flushes every g, hybrids switching at launch 5 / 17
SCHEDULES = ((0, 1, -1), (1, 1, -1), (1, 4, -1), (1, 6, -1), (1, 8, -1), (-1, 2, 5), (-1, 4, 17))


@pytest.mark.parametrize("n", [4096, 8320])
def test_fit_bits_identical_across_schedules_and_batches(engine, n):
    """Schedule-invariant arithmetic (gpx_potrf.hip trailing_tile_at): every trailing-update actor seeds its accumulator
    with the matrix entry and adds the products of the pending columns in their k order, so L, z and alpha do not depend
    on how the launches group the columns.  The default single fit (n = 4096: lookahead start then eager; n = 8320:
    lookahead then the eager tail), every forced schedule and the default batched fits (lookahead, g = 4 / 6 / 8, panels
    split by the slots a problem gets) give the same bits.  This is what makes a restart's result independent of how
    restarts are split over GPUs (BASELINE configs[3]; selection site /root/reference/optimization/Bayesian.py:105-112)."""
    X, y = O.synthetic_problem(n, 8, 40)
    kp, _ = pair("rbf", 8, noise=1e-4)
    ref = engine.fit(t(X), t(y), kp)
    L0, a0 = torch.tril(ref.L).clone(), ref.alpha.clone()
    del ref
    for mode, lazy, sw in SCHEDULES:
        engine.set_option("potrf_mode", mode)
        engine.set_option("potrf_lazy", lazy)
        engine.set_option("potrf_switch", sw)
        try:
            st = engine.fit(t(X), t(y), kp)
        finally:
            engine.set_option("potrf_mode", -1)
            engine.set_option("potrf_lazy", 0)
            engine.set_option("potrf_switch", -1)
        assert torch.equal(torch.tril(st.L), L0), (mode, lazy, sw)
        assert torch.equal(st.alpha, a0), (mode, lazy, sw)
        del st
    for B in ((2, 4) if n == 4096 else (2,)):
        sts = engine.fit_batched(t(np.stack([X] * B)), t(np.stack([y] * B)), kp)
        for s in sts:
            assert torch.equal(torch.tril(s.L), L0), B
            assert torch.equal(s.alpha, a0), B
        del sts


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


@pytest.mark.parametrize("nrhs", [1, 8])
@pytest.mark.parametrize("batch", [1, 3])
def test_lookahead_schedule_folded_alpha_vs_oracle(engine, nrhs, batch):
    """The forward substitution folded into the LOOKAHEAD panel schedule (potrf_mode 1, the default for padded n > 4096)
    at a small size: alpha of the default update against the oracle, single and batched, 1 and 8 right-hand sides
    (only the eager schedule was compared below n = 8192)."""
    n, d = 1000, 5
    kp, op = pair("rbf", d, noise=1e-3, const_mean=0.1)
    probs = [O.synthetic_problem(n, d, 60 + b) for b in range(batch)]
    Ys = [np.stack([yb * (r + 1) - 0.2 * r for r in range(nrhs)], 1) for _, yb in probs]
    for mode, lazy in ((1, 1), (1, 3)):
        engine.set_option("potrf_mode", mode)
        engine.set_option("potrf_lazy", lazy)
        try:
            if batch == 1:
                sts = [engine.fit(t(probs[0][0]), t(Ys[0]), kp)]
            else:
                sts = engine.fit_batched(t(np.stack([Xb for Xb, _ in probs])), t(np.stack(Ys)), kp)
        finally:
            engine.set_option("potrf_mode", -1)
            engine.set_option("potrf_lazy", 0)
        for b, st in enumerate(sts):
            a = st.alpha.cpu().numpy()
            ar = O.fit(probs[b][0], Ys[b], op).alpha.reshape(n, nrhs)
            assert np.abs(a[:n] - ar).max() <= 1e-8 * np.abs(ar).max(), (mode, lazy, b)
            assert not np.any(a[n:])


def test_standalone_potrs_timeout_leaves_state_valid(engine):
    """A timed-out standalone solve (new targets on a fitted factor) raises GPXTimeoutError from its own info word; the
    fitted state keeps info 0, its alpha and its posterior."""
    n = 2048
    X, y = O.synthetic_problem(n, 8, 24)
    kp, _ = pair("rbf", 8, noise=1e-4)
    st = engine.fit(t(X), t(y), kp)
    alpha0 = st.alpha.clone()
    # the standalone solve runs its own forward substitution (the fit folds it into the Cholesky): a different summation
    # order, so its reference is a standalone solve of y (scaling the targets by 0.5 is exact)
    a_ref = engine.potrs(st, t(y))
    engine.set_option("spin_limit", 0)
    try:
        with pytest.raises(GPXTimeoutError):
            engine.potrs(st, t(y * 0.5))
    finally:
        engine.set_option("spin_limit", 1 << 22)
    assert int(st.info.item()) == 0 and st.pivot_failure() == -1
    assert torch.equal(st.alpha, alpha0)
    a2 = engine.potrs(st, t(y * 0.5))
    assert torch.equal(a2, a_ref * 0.5)
    assert float((a2 - alpha0 * 0.5).abs().max()) <= 1e-9 * float(alpha0.abs().max())


def test_fit_beside_a_long_kernel_on_another_stream(engine):
    """the backward solve is one persistent launch whose hand-offs assume its workgroups become
    resident.  With torch DGEMMs (~100 ms) queued on a second stream first, so that they hold CUs while the fit's
    launches arrive, the fit must either complete with the same alpha bit for bit or raise GPXTimeoutError - never
    return NaN or a wrong alpha silently."""
    n = 4096
    X, y = O.synthetic_problem(n, 8, 25)
    kp, _ = pair("rbf", 8, noise=1e-4)
    ref = engine.fit(t(X), t(y), kp)
    alpha_ref = ref.alpha.clone()
    side = torch.cuda.Stream(device=engine.device)
    A = torch.randn(6144, 6144, dtype=torch.float64, device=engine.device) / 6144 ** 0.5
    torch.cuda.synchronize()
    outcomes = []
    for _ in range(3):
        with torch.cuda.stream(side):
            B = A
            for _ in range(8):
                B = A @ B
        try:
            st = engine.fit(t(X), t(y), kp)
            torch.cuda.synchronize()
            assert torch.isfinite(st.alpha).all()
            assert torch.equal(st.alpha, alpha_ref)
            outcomes.append("ok")
        except GPXTimeoutError:
            torch.cuda.synchronize()
            outcomes.append("timeout")
    # the timeout rate under contention, visible in the test log; ExactGP.fit turns a timeout into a
    # refit through the hand-off-free path (tests/test_dropin_gpu.py::test_dropin_survives_timed_out_handoffs)
    print(f"contention outcomes: {outcomes}")
    assert outcomes.count("ok") >= 1, f"contention outcomes: {outcomes}"
