"""Multi-GPU sharding of independent GP problems, one process per GPU.

Independent units — restarts / seeds / outputs (BASELINE configs[3]: 32 x n=4096 over 8 GPUs) or contiguous
candidate shards of one large sweep — are partitioned in contiguous blocks across ranks; every rank fits
and sweeps its own units with no data-path collective.  The single exchange is one 16-byte
(fp64 value, int64 global index) record per rank: on an nccl group ONE RCCL all-gather through libgpx's own
communicator (gpx_allreduce_argmax) followed by the deterministic argmax_combine kernel (max value, then lowest global
index; RCCL has no MAXLOC op, hence gather + local reduce); on gloo the same packed records and the same reduction order
on the host.  Reference selection site: optimization/Bayesian.py:105-112 (best restart of optimize_acqf).
"""
from __future__ import annotations

import ctypes
from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def shard_range(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous block partition: rank r gets [start, stop) with sizes differing by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("invalid rank/world")
    q, r = divmod(total, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def pack_record(val: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """The 16-byte exchange record {fp64 value; int64 global index} as two int64 words, exactly as libgpx's
    record_pack_kernel writes it (gpx_sweep.hip): word 0 = the value's bit pattern, word 1 = the index."""
    v = val.reshape(1).to(torch.float64).cpu()
    i = idx.reshape(1).to(torch.int64).cpu()
    return torch.cat([v.view(torch.int64), i])


def unpack_records(recs: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(values, indices) of a (count, 2) int64 record array."""
    recs = recs.reshape(-1, 2).contiguous()
    return recs[:, 0].contiguous().view(torch.float64), recs[:, 1].contiguous()


def combine_records_host(vals: torch.Tensor, idx: torch.Tensor) -> Tuple[float, int]:
    """Host reduction in the device kernel's order (argmax_final_kernel, gpx_sweep.hip): start from (-inf, INT64_MAX),
    NaN counts as -inf, a record wins with a larger value or an equal value and a lower index."""
    best_v, best_i = float("-inf"), 2 ** 63 - 1
    for v, i in zip(vals.reshape(-1).tolist(), idx.reshape(-1).tolist()):
        if v != v:  # NaN never wins
            v = float("-inf")
        if v > best_v or (v == best_v and i < best_i):
            best_v, best_i = v, i
    return best_v, best_i


def _rccl_exchange(engine, group) -> "RCCLArgmaxExchange":
    """libgpx's communicator for (engine, group), created on first use (collective: every rank of the group calls
    exchange_argmax together, as the exchange itself requires)."""
    cache = engine.__dict__.setdefault("_rccl_exchanges", {})
    key = id(group) if group is not None else None
    ex = cache.get(key)
    if ex is None:
        ex = RCCLArgmaxExchange(engine, group)
        cache[key] = ex
    return ex


def exchange_argmax(val: torch.Tensor, idx: torch.Tensor, engine=None, group=None):
    """Every rank's (value, global index) record -> the global best, with ONE collective per call.

    nccl group (GPU records): libgpx's RCCL communicator (RCCLArgmaxExchange, gpx_allreduce_argmax): one all-gather
    of the 16-byte records over xGMI and the deterministic argmax_combine kernel on the engine's stream — the path
    bench.py --gpus N runs.  gloo group (CPU tests): one all-gather of the same packed records, reduced by the host loop
    in the kernel's order.  Returns (value, index) as 1-element tensors on val's device."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    val = val.reshape(1).to(torch.float64)
    idx = idx.reshape(1).to(torch.int64)
    if world == 1:
        return val, idx
    if dist.get_backend(group) == "nccl":
        if engine is None or not val.is_cuda:
            raise ValueError("the RCCL record exchange needs device records and the engine that owns the communicator")
        v, i = val.clone(), idx.clone()
        _rccl_exchange(engine, group)(v, i)
        return v, i
    recs = [torch.empty(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(recs, pack_record(val, idx), group=group)
    v, i = combine_records_host(*unpack_records(torch.stack(recs)))
    return (torch.tensor([v], dtype=torch.float64, device=val.device),
            torch.tensor([i], dtype=torch.int64, device=val.device))


def sharded_best(num_units: int, local_best: Callable[[int], Tuple[torch.Tensor, torch.Tensor]],
                 engine=None, group=None):
    """Run ``local_best(unit)`` for this rank's contiguous share of ``num_units`` independent problems;
    each returns (value, global_index) for its unit.  Reduce locally, then across ranks.

    Returns (value, index, unit_results) where unit_results lists this rank's (unit, value, index).
    """
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    start, stop = shard_range(num_units, rank, world)
    vals: List[torch.Tensor] = []
    idxs: List[torch.Tensor] = []
    results = []
    for u in range(start, stop):
        v, i = local_best(u)
        vals.append(v.reshape(1).to(torch.float64))
        idxs.append(i.reshape(1).to(torch.int64))
        results.append((u, v, i))
    if vals:
        lv, li = torch.cat(vals), torch.cat(idxs)
        if engine is not None and lv.is_cuda:
            bv, bi = engine.argmax_combine(lv, li)
        else:
            v, i = combine_records_host(lv, li)
            bv = torch.tensor([v], dtype=torch.float64, device=lv.device)
            bi = torch.tensor([i], dtype=torch.int64, device=lv.device)
    else:  # more ranks than units
        dev = torch.device("cuda", torch.cuda.current_device()) if engine is not None else torch.device("cpu")
        bv = torch.tensor([float("-inf")], dtype=torch.float64, device=dev)
        bi = torch.tensor([2 ** 63 - 1], dtype=torch.int64, device=dev)
    v, i = exchange_argmax(bv, bi, engine=engine, group=group)
    return v, i, results


def sharded_sweep(engine, state, Xs: torch.Tensor, kind: str = "logei", group=None, **acq_kwargs):
    """One fit, many candidates: every rank holds the same fitted ``state`` (the factorisation
    is recomputed on each GPU — ~2.5 ms at n = 4096, cheaper than broadcasting 128 MiB of L) and scores its
    contiguous shard [start, stop) of the global candidate set ``Xs`` (m x d, identical on every rank); the
    (value, global index) records are then exchanged once.  Returns (value, index) 1-element tensors."""
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    start, stop = shard_range(Xs.shape[0], rank, world)
    if stop > start:
        bv, bi = engine.acquire(state, Xs[start:stop], kind, index_offset=start, **acq_kwargs)
    else:
        dev = Xs.device
        bv = torch.tensor([float("-inf")], dtype=torch.float64, device=dev)
        bi = torch.tensor([2 ** 63 - 1], dtype=torch.int64, device=dev)
    return exchange_argmax(bv, bi, engine=engine, group=group)


class RCCLArgmaxExchange:
    """The record exchange through libgpx's own RCCL communicator (gpx_allreduce_argmax, include/gpx.h): rank 0 makes
    the communicator id, torch.distributed broadcasts its 128 bytes once, then every exchange is one RCCL all-gather
    of the 16-byte records plus the argmax_combine kernel on the engine's stream — no torch collective on the hot
    path.  ``__call__(val, idx)`` replaces the device records in place by the global best and returns them."""

    def __init__(self, engine, group=None):
        from . import _capi

        self.engine = engine
        self.lib = engine.lib
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        buf = (ctypes.c_ubyte * _capi.GPX_COMM_ID_BYTES)()
        if rank == 0:
            _capi.check(self.lib.gpx_comm_unique_id(ctypes.cast(buf, ctypes.c_void_p)))
        if world > 1:
            backend = dist.get_backend(group)
            dev = engine.device if backend == "nccl" else torch.device("cpu")
            t = torch.tensor(list(buf), dtype=torch.uint8, device=dev)
            dist.broadcast(t, src=0, group=group)
            for k, v in enumerate(t.cpu().tolist()):
                buf[k] = v
        self.comm = ctypes.c_void_p()
        _capi.check(self.lib.gpx_comm_init(engine.handle, ctypes.cast(buf, ctypes.c_void_p), world, rank,
                                           ctypes.byref(self.comm)), engine.handle)
        nbytes = ctypes.c_size_t()
        _capi.check(self.lib.gpx_allreduce_argmax_workspace_size(self.comm, ctypes.byref(nbytes)))
        self.ws = torch.empty(nbytes.value, dtype=torch.uint8, device=engine.device)

    def __call__(self, val: torch.Tensor, idx: torch.Tensor):
        from . import _capi

        if val.dtype != torch.float64 or idx.dtype != torch.int64 or not val.is_cuda or val.numel() != 1 \
                or idx.numel() != 1:
            raise ValueError("records must be 1-element fp64 / int64 device tensors")
        self.engine._bind_stream()
        _capi.check(self.lib.gpx_allreduce_argmax(self.engine.handle, self.comm, ctypes.c_void_p(val.data_ptr()),
                                                  ctypes.c_void_p(idx.data_ptr()),
                                                  ctypes.c_void_p(self.ws.data_ptr()), self.ws.numel()),
                    self.engine.handle)
        return val, idx

    def close(self):
        if self.comm:
            self.lib.gpx_comm_destroy(self.comm)
            self.comm = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
