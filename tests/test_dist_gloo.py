"""World-size-2 gloo tests of the multi-GPU path's host logic: contiguous sharding of independent
problems and the (value, index) exchange.  Each rank computes its units with the CPU oracle standing in for the
device engine; the exchange and reduction code is the product's (bayesianoptimizer_amd.dist)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _oracle_unit_best(unit, m=300, n=64, d=3):
    from oracle import gp_oracle as O

    X, y = O.synthetic_problem(n, d, 100 + unit)
    Xs = O.sobol_candidates(m, d, 500 + unit)
    st = O.fit(X, y, O.KernelParams(O.RBF, np.full(d, 0.4), noise=1e-4))
    v, i, _ = O.acquire_argmax(st, Xs, O.ACQ_LOGEI, best_f=float(y.max()))
    return v, unit * m + i


def _worker(rank, world, port, num_units, q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bayesianoptimizer_amd.dist import exchange_argmax, sharded_best

        def local_best(u):
            v, i = _oracle_unit_best(u)
            return torch.tensor([v], dtype=torch.float64), torch.tensor([i], dtype=torch.int64)

        v, i, res = sharded_best(num_units, local_best)
        # explicit exchange with a deliberate tie: every rank offers value 1.0 with index 10 - rank
        tv, ti = exchange_argmax(torch.tensor([1.0], dtype=torch.float64), torch.tensor([10 - rank]))
        q.put((rank, float(v), int(i), [u for u, _, _ in res], float(tv), int(ti)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("num_units", [5, 1])
def test_sharded_best_world2(num_units):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, num_units, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    # every rank agrees on the global best
    assert out[0][1:3] == out[1][1:3]
    # contiguous partition of the units
    assert out[0][3] + out[1][3] == list(range(num_units))
    # matches a serial reduction over all units
    from oracle import gp_oracle as O

    best = O.combine_argmax([_oracle_unit_best(u) for u in range(num_units)])
    assert out[0][1] == pytest.approx(best[0], rel=0, abs=0) and out[0][2] == best[1]
    # tie -> lowest index (rank 1 offered index 9)
    assert out[0][4:] == (1.0, 9) and out[1][4:] == (1.0, 9)


def _sweep_worker(rank, world, port, m, q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bayesianoptimizer_amd.dist import sharded_sweep
        from bayesianoptimizer_amd.engine import KernelParams
        from oracle import gp_oracle as O
        from tests.oracle_engine import OracleEngine

        X, y = O.synthetic_problem(80, 3, 4)
        Xs = torch.tensor(O.sobol_candidates(m, 3, 5))
        eng = OracleEngine()
        st = eng.fit(torch.tensor(X), torch.tensor(y), KernelParams("rbf", 0.4, noise=1e-4))
        v, i = sharded_sweep(eng, st, Xs, "logei", best_f=float(y.max()))
        q.put((rank, float(v), int(i)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,m", [(2, 1000), (3, 2)])
def test_sharded_sweep_one_fit_many_candidates(world, m):
    # the same fit on every rank, contiguous candidate shards, one record exchange
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sweep_worker, args=(r, world, port, m, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle import gp_oracle as O

    X, y = O.synthetic_problem(80, 3, 4)
    st = O.fit(X, y, O.KernelParams(O.RBF, np.full(3, 0.4), noise=1e-4))
    v_ref, i_ref, _ = O.acquire_argmax(st, O.sobol_candidates(m, 3, 5), O.ACQ_LOGEI, best_f=float(y.max()))
    for _, v, i in out:
        assert i == i_ref and v == pytest.approx(v_ref, rel=1e-10)  # shard vs full-set BLAS blocking


# ---- the record exchange itself: one packed 16-byte record per rank, one collective -------------------------------
def _device_combine(records):
    """Restatement of libgpx's argmax_final_kernel over packed records (gpx_sweep.hip): (-inf, INT64_MAX) start, NaN
    counts as -inf, a larger value wins, an equal value with a lower index wins."""
    bv, bi = float("-inf"), 2 ** 63 - 1
    for word0, idx in records:
        v = float(np.array([word0], dtype=np.int64).view(np.float64)[0])
        if v != v:
            v = float("-inf")
        if v > bv or (v == bv and idx < bi):
            bv, bi = v, idx
    return bv, bi


def test_pack_record_matches_record_pack_kernel_layout():
    from bayesianoptimizer_amd.dist import pack_record, unpack_records

    for v, i in ((1.5, 7), (-0.0, 0), (float("inf"), 2 ** 62), (float("nan"), 3), (-1e-300, 2 ** 63 - 1)):
        rec = pack_record(torch.tensor([v], dtype=torch.float64), torch.tensor([i]))
        # struct {double value; int64_t index} of record_pack_kernel: value bits, then index
        raw = np.frombuffer(np.array([v], dtype=np.float64).tobytes() + np.array([i], dtype=np.int64).tobytes(),
                            dtype=np.int64)
        assert rec.tolist() == raw.tolist()
        vv, ii = unpack_records(rec)
        assert (vv.item() == v or (v != v and vv.item() != vv.item())) and ii.item() == i


def test_host_combine_follows_device_order_random():
    from bayesianoptimizer_amd.dist import combine_records_host, pack_record

    rng = np.random.default_rng(3)
    pool = [0.5, -2.0, float("inf"), float("-inf"), float("nan"), 0.5, 1e300]
    for trial in range(300):
        k = int(rng.integers(1, 9))
        vals = [pool[int(rng.integers(len(pool)))] for _ in range(k)]
        idxs = [int(rng.integers(0, 6)) for _ in range(k)]
        recs = [pack_record(torch.tensor([v], dtype=torch.float64), torch.tensor([i])).tolist() for v, i in zip(vals, idxs)]
        hv, hi = combine_records_host(torch.tensor(vals, dtype=torch.float64), torch.tensor(idxs))
        dv, di = _device_combine(recs)
        assert (hv, hi) == (dv, di), (vals, idxs)


def _exchange_worker(rank, world, port, cases, q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bayesianoptimizer_amd.dist as D

        calls = {"all_gather": 0, "other": 0}
        real_all_gather = dist.all_gather

        def counting_all_gather(*a, **kw):
            calls["all_gather"] += 1
            return real_all_gather(*a, **kw)

        D.dist.all_gather = counting_all_gather
        D.dist.all_gather_into_tensor = lambda *a, **kw: calls.__setitem__("other", calls["other"] + 1)
        out = []
        for case in cases:
            v, i = case[rank]
            before = calls["all_gather"]
            bv, bi = D.exchange_argmax(torch.tensor([v], dtype=torch.float64), torch.tensor([i]))
            out.append((float(bv), int(bi), calls["all_gather"] - before))
        q.put((rank, out, calls["other"]))
    finally:
        dist.destroy_process_group()


def test_exchange_one_collective_nan_and_ties_world2():
    """Each exchange is ONE all-gather of packed 16-byte records (never a value gather plus an index gather); every
    rank reaches the device kernel's answer, NaN never wins, ties go to the lowest global index."""
    nan = float("nan")
    cases = [
        [(nan, 3), (1.0, 7)],            # NaN loses to anything
        [(2.0, 9), (2.0, 4)],            # tie -> lowest index
        [(nan, 5), (nan, 2)],            # all NaN -> (-inf, lowest index)
        [(float("-inf"), 1), (-5.0, 8)],
        [(3.0, 2 ** 40), (3.0, 2 ** 40 + 1)],
    ]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, 2, port, cases, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from bayesianoptimizer_amd.dist import pack_record

    for rank, res, other in out:
        assert other == 0
        for case, (v, i, ncoll) in zip(cases, res):
            recs = [pack_record(torch.tensor([cv], dtype=torch.float64), torch.tensor([ci])).tolist() for cv, ci in case]
            assert (v, i) == _device_combine(recs)
            assert ncoll == 1
