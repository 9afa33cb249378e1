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
