"""Benchmark of the GP-posterior hot path (BASELINE.json metric), one process per GPU.

A step = one posterior update (Gram + blocked Cholesky + alpha by triangular solves, n=4096, d=8, RBF, fp64;
SURVEY §8d's unit) followed by a 2^20-candidate analytic logEI sweep with argmax (BASELINE.json configs[1]) —
which first builds the explicit inverse L^{-T} its triangular product needs — then the cross-rank (value, index)
exchange.  Every rank owns an independent problem (different seed: weak scaling); the
only collective is an all-gather of one 16-byte record per rank over RCCL.

Prints ONE JSON line on rank 0.  value = candidates scored per second over the whole job
(= n_gpus * m * steps / max-over-ranks time); the fit-only rate (posterior updates/s) is timed in a second
loop and reported beside it.  Inputs are resident in HBM before the timed region starts.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       N>1 either under a launcher (python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ...
       bench.py --gpus N: WORLD_SIZE must equal N) or bare: `python bench.py --gpus N` then starts the N ranks itself
       (launch_ranks) before anything in this process touches the GPU, so n_gpus = N by construction.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from bayesianoptimizer_amd import GPEngine, KernelParams, botorch_default_lengthscale, synthetic  # noqa: E402
from bayesianoptimizer_amd.dist import RCCLArgmaxExchange  # noqa: E402

METRIC = "GP posterior updates/sec + acq-cands/sec, n=4096 d=8 fp64, 1→8 MI355X"
FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 matrix, spec; measured 78.1 TF/s (profiles/r01_probe_f64_rate.log)
HBM_PEAK_GBS = 8000.0


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--d", type=int, default=8)
    ap.add_argument("--m", type=int, default=1 << 20)
    ap.add_argument("--kernel", default="rbf")
    ap.add_argument("--acq", default="logei")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--problems-per-gpu", type=int, default=1,
                    help="independent problems (restarts/seeds) per GPU per step; 4 at 8 GPUs = BASELINE configs[3]")
    ap.add_argument("--cpu-sample", type=int, default=8192, help="candidates in the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="skip the side measurements of BASELINE configs[2] and configs[4] (N=1 only)")
    ap.add_argument("--launcher-selftest", action="store_true",
                    help="test hook: every rank reports its rank variables and exits before any GPU call")
    return ap.parse_args(argv)


def launch_ranks(gpus: int, argv) -> int:
    """`bench.py --gpus N` without a launcher around it: run N ranks of this script under torch.distributed.run
    (one process per GPU, rendezvous on 127.0.0.1, a free port) as a CHILD process and return its exit status.  Called
    before this process makes any HIP call (no GPEngine, no torch.cuda query): the children own the GPUs."""
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")  # torch.distributed.run's default for N > 1, stated to keep it quiet
    return subprocess.call(cmd, env=env)


def check_world(args) -> None:
    """Under a launcher the world it started must be the one --gpus names (the driver passes both)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; launch N ranks for --gpus N "
                         f"(or run bare: bench.py --gpus N starts them itself)")


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        return dist, rank, world, local
    torch.cuda.set_device(0)
    return None, 0, 1, 0


def barrier(dist):
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()


PMC_TRAFFIC_FILE = os.path.join("profiles", "trmm_pmc_traffic.json")


def pmc_traffic_record():
    """HBM bytes per trmm launch from the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic.py; the
    round check runs them right before this bench on the same box and tree), and where that number came from."""
    path = os.path.join(ROOT, PMC_TRAFFIC_FILE)
    if not os.path.exists(path):
        return None, None
    try:
        with open(path) as f:
            rec = json.load(f)
    except Exception:
        return None, None
    # "recorded": read from the PMC passes' file, not measured by this process (rocprofv3 --pmc cannot run inside it);
    # the evidence script regenerates the file in the same call, on the same box and tree, right before its bench line
    src = {"kind": "recorded", "file": PMC_TRAFFIC_FILE, "generated_utc": rec.get("generated_utc"),
           "dispatches": rec.get("dispatches"), "passes": rec.get("passes")}
    return rec.get("hbm_bytes_per_launch"), src


def _torch_cpu_step(X, y, Xs, ls, noise, best_f, kind):
    """The same posterior update + logEI sweep in torch-CPU fp64 (MKL/OpenBLAS LAPACK): Gram, Cholesky,
    alpha, then per 4096-candidate block k*, mu, V = L^-1 k*, var, score, running argmax."""
    from oracle import gp_oracle as O  # logEI helper (checker code, baseline leg only)

    Xt = torch.from_numpy(X) / ls

    def cov(A, B):
        r2 = torch.cdist(A, B).square_()
        if kind == "rbf":
            return torch.exp(-0.5 * r2)
        r = r2.sqrt()
        return (1.0 + 5.0 ** 0.5 * r + (5.0 / 3.0) * r2) * torch.exp(-(5.0 ** 0.5) * r)

    K = cov(Xt, Xt)
    K.diagonal().add_(noise)
    L = torch.linalg.cholesky(K)
    alpha = torch.cholesky_solve(torch.from_numpy(y).reshape(-1, 1), L)
    best = (-float("inf"), -1)
    for s0 in range(0, Xs.shape[0], 4096):
        Xc = torch.from_numpy(Xs[s0:s0 + 4096]) / ls
        Ks = cov(Xt, Xc)  # n x c
        mu = (Ks.T @ alpha).reshape(-1)
        V = torch.linalg.solve_triangular(L, Ks, upper=False)
        var = torch.clamp(1.0 - V.square().sum(0), min=1e-12)
        sd = var.sqrt()
        sc = O.log_ei_helper(((mu - best_f) / sd).numpy()) + np.log(sd.numpy())
        i = int(np.argmax(sc))
        if sc[i] > best[0]:
            best = (float(sc[i]), s0 + i)
    return best


def cpu_baseline(X, y, Xs_np, kind, acq, ls, sample, reps=5):
    """CPU baseline on the host cores, two restatements of the same step, the faster one reported:
    the NumPy/SciPy oracle (one fit + a sweep over `sample` candidates) and torch-CPU fp64 (median of `reps`
    after a warm-up, over 8x the sample).  Each is extrapolated linearly from its sample to the full step."""
    from oracle import gp_oracle as O  # checker / baseline only

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    torch.set_num_threads(threads)
    m = Xs_np.shape[0]
    kid = {"rbf": O.RBF, "matern52": O.MATERN52, "scale_linear_matern52": O.SCALE_LINEAR_MATERN52}[kind]
    aid = {"ei": O.ACQ_EI, "logei": O.ACQ_LOGEI, "ucb": O.ACQ_UCB, "variance": O.ACQ_VARIANCE}[acq]
    p = O.KernelParams(kid, np.full(X.shape[1], ls), noise=1e-4)
    t0 = time.perf_counter()
    st = O.fit(X, y, p)
    t1 = time.perf_counter()
    O.acquire_argmax(st, Xs_np[:sample], aid, best_f=float(y.max()), chunk=4096)
    t2 = time.perf_counter()
    oracle_step = (t1 - t0) + (t2 - t1) * (m / sample)
    cands = [{"value": m / oracle_step, "what": f"NumPy/SciPy oracle: fit {t1 - t0:.2f} s + {acq} sweep of {sample} "
                                                  f"candidates {t2 - t1:.2f} s"}]
    if acq == "logei" and kind in ("rbf", "matern52"):
        ts = 8 * sample
        times = []
        for r in range(reps + 1):
            a = time.perf_counter()
            _torch_cpu_step(X, y, Xs_np[:ts], ls, 1e-4, float(y.max()), kind)
            times.append(time.perf_counter() - a)
        tt = float(np.median(times[1:]))
        # fit share measured separately so the extrapolation scales only the sweep
        a = time.perf_counter()
        _torch_cpu_step(X, y, Xs_np[:1], ls, 1e-4, float(y.max()), kind)
        tfit = time.perf_counter() - a
        torch_step = tfit + max(tt - tfit, 0.0) * (m / ts)
        cands.append({"value": m / torch_step, "what": f"torch-CPU fp64: fit {tfit:.2f} s, fit + {ts}-candidate "
                                                       f"sweep median {tt:.2f} s over {reps} reps"})
    best = max(cands, key=lambda c: c["value"])
    return {"value": best["value"], "unit": "acq-cands/s", "cores": threads, "kind": "port",
            "sample": f"{best['what']}; extrapolated linearly to one full {m}-candidate step (n={X.shape[0]}); "
                      f"faster of: " + "; ".join(f"{c['what'].split(':')[0]} {c['value']:.4g}" for c in cands)}


def other_configs(eng, dev, seed):
    """Side measurements at N=1 of the other GPU configs of BASELINE.json (not the headline `value`):
    configs[2] n=16384 d=8 Matern-5/2 posterior update and a whole n = 16384 step (update + L^-T + 2^20-candidate
    logEI sweep), configs[4] n=4096 d=16 fp32 covariance build + UCB sweep, and the north star's n = 1024 point
    (update + EI sweep)."""
    out = {}
    X_np, y_np = synthetic.problem(16384, 8, seed + 7)
    X, y = torch.tensor(X_np, device=dev), torch.tensor(y_np, device=dev)
    p = KernelParams("matern52", botorch_default_lengthscale(8), noise=1e-4)
    st = eng.fit(X, y, p)
    ts = []
    for _ in range(3):
        torch.cuda.synchronize()
        a = time.perf_counter()
        st = eng.fit(X, y, p, check=False, out=st)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - a)
    if st.pivot_failure() >= 0:
        raise RuntimeError("configs[2] Cholesky failed")
    t = float(np.median(ts))
    torch.cuda.synchronize()
    a = time.perf_counter()
    eng.inverse(st)  # what the first sweep after this update would add
    torch.cuda.synchronize()
    ti = time.perf_counter() - a
    out["configs[2]"] = {"workload": "n=16384 d=8 Matern-5/2 fp64 posterior update (Gram + Cholesky + alpha by "
                                     "triangular solves)", "fit_ms": 1e3 * t, "updates_per_s": 1.0 / t,
                         "update_tflops_n3_over_3": 16384.0 ** 3 / 3 / t / 1e12,
                         "inverse_ms_for_a_following_sweep": 1e3 * ti}
    # the north star's n = 16k point for the acquisition rate: one whole step at configs[2]'s model, i.e. the posterior
    # update, the L^-T its sweep needs and a 2^20-candidate logEI sweep + argmax (after one untimed step)
    Xs16 = torch.tensor(synthetic.sobol(1 << 20, 8, seed + 8), device=dev)
    bf16 = float(y_np.max())

    def step16():
        s16 = eng.fit(X, y, p, check=False, out=st)
        return eng.acquire(s16, Xs16, "logei", best_f=bf16)

    step16()
    torch.cuda.synchronize()
    eng.timing_reset()
    eng.timing_enable(["trmm"])
    a = time.perf_counter()
    bv, bi = step16()
    torch.cuda.synchronize()
    t16 = time.perf_counter() - a
    trmm16_ms, trmm16_n = eng.timing_query("trmm")
    eng.timing_disable()
    if st.pivot_failure() >= 0:
        raise RuntimeError("n=16384 sweep: Cholesky failed")
    chunk16 = (1 << 20) / max(trmm16_n, 1)
    trmm16_tf = 16384.0 ** 2 * chunk16 / (trmm16_ms / max(trmm16_n, 1) * 1e-3) / 1e12
    out["n=16384 sweep"] = {"workload": "n=16384 d=8 Matern-5/2 fp64: posterior update + L^-T + 1048576-candidate "
                                        "logEI sweep + argmax (one step)", "ms_per_step": 1e3 * t16,
                            "acq_cands_per_s": (1 << 20) / t16, "trmm_tflops": trmm16_tf,
                            "trmm_frac": trmm16_tf / FP64_PEAK_TFLOPS, "trmm_launches": trmm16_n,
                            "best_index": int(bi.item())}
    del st, X, y, Xs16
    torch.cuda.empty_cache()
    X_np, y_np = synthetic.problem(4096, 16, seed + 11)
    Xs_np = synthetic.sobol(1 << 20, 16, seed + 12)
    X, y, Xs = (torch.tensor(v, device=dev) for v in (X_np, y_np, Xs_np))
    p = KernelParams("rbf", botorch_default_lengthscale(16), noise=1e-4, cov_fp32=True)
    st = eng.fit(X, y, p)
    eng.acquire(st, Xs, "ucb", beta=4.0)
    ts = []
    for _ in range(2):
        torch.cuda.synchronize()
        a = time.perf_counter()
        st = eng.fit(X, y, p, check=False, out=st)
        bv, bi = eng.acquire(st, Xs, "ucb", beta=4.0)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - a)
    t = float(np.median(ts))
    out["configs[4]"] = {"workload": "n=4096 d=16 RBF, fp32 covariance build, fp64 factorisation, 1048576-candidate "
                                     "UCB sweep + argmax", "ms_per_step": 1e3 * t, "acq_cands_per_s": (1 << 20) / t,
                         "best_index": int(bi.item())}
    del st, X, y, Xs
    torch.cuda.empty_cache()
    # the north star's n = 1k point (n in {1k, 4k, 16k}): posterior update + 2^20-candidate EI sweep + argmax
    X_np, y_np = synthetic.problem(1024, 8, seed + 13)
    Xs_np = synthetic.sobol(1 << 20, 8, seed + 14)
    X, y, Xs = (torch.tensor(v, device=dev) for v in (X_np, y_np, Xs_np))
    p = KernelParams("rbf", botorch_default_lengthscale(8), noise=1e-4)
    bf = float(y_np.max())
    st = eng.fit(X, y, p)
    eng.acquire(st, Xs, "ei", best_f=bf)
    tf, ts = [], []
    for _ in range(3):
        torch.cuda.synchronize()
        a = time.perf_counter()
        st = eng.fit(X, y, p, check=False, out=st)
        torch.cuda.synchronize()
        b = time.perf_counter()
        bv, bi = eng.acquire(st, Xs, "ei", best_f=bf)
        torch.cuda.synchronize()
        tf.append(b - a)
        ts.append(time.perf_counter() - a)
    t, f = float(np.median(ts)), float(np.median(tf))
    out["n=1024"] = {"workload": "n=1024 d=8 RBF fp64 posterior update + 1048576-candidate EI sweep + argmax",
                     "fit_ms": 1e3 * f, "updates_per_s": 1.0 / f, "ms_per_step": 1e3 * t,
                     "acq_cands_per_s": (1 << 20) / t, "best_index": int(bi.item())}
    del st, X, y, Xs
    torch.cuda.empty_cache()
    # configs[0]'s problem size (n = 256 d = 4 RBF EI, the reference's own CPU case) on the GPU: the fused small-n
    # sweep (sweep_small_kernel) over 2^20 candidates, plus its posterior update
    X_np, y_np = synthetic.problem(256, 4, seed + 15)
    Xs_np = synthetic.sobol(1 << 20, 4, seed + 16)
    X, y, Xs = (torch.tensor(v, device=dev) for v in (X_np, y_np, Xs_np))
    p = KernelParams("rbf", botorch_default_lengthscale(4), noise=1e-4)
    bf = float(y_np.max())
    st = eng.fit(X, y, p)
    eng.acquire(st, Xs, "ei", best_f=bf)
    tf, ts = [], []
    for _ in range(5):
        torch.cuda.synchronize()
        a = time.perf_counter()
        st = eng.fit(X, y, p, check=False, out=st)
        torch.cuda.synchronize()
        b = time.perf_counter()
        bv, bi = eng.acquire(st, Xs, "ei", best_f=bf)
        torch.cuda.synchronize()
        tf.append(b - a)
        ts.append(time.perf_counter() - b)
    f, s = float(np.median(tf)), float(np.median(ts))
    out["n=256 (configs[0] size)"] = {
        "workload": "n=256 d=4 RBF fp64 posterior update; 1048576-candidate EI sweep + argmax (fused small-n sweep)",
        "fit_ms": 1e3 * f, "updates_per_s": 1.0 / f, "sweep_ms": 1e3 * s, "acq_cands_per_s": (1 << 20) / s,
        "best_index": int(bi.item())}
    del st, X, y, Xs
    torch.cuda.empty_cache()
    # BASELINE configs[3] at its per-GPU share (32 restarts over 8 GPUs = 4 per GPU): 4 independent n = 4096 d = 8 RBF
    # problems fitted in the same launches (gpx_fit_batched_f64), a 2^20-candidate logEI sweep each and the local
    # combine of their records (the cross-GPU exchange is the --gpus N path of the headline line)
    P4 = 4
    pr = [synthetic.problem(4096, 8, seed + 100 + q) for q in range(P4)]
    Xb = torch.tensor(np.stack([a for a, _ in pr]), device=dev)
    yb = torch.tensor(np.stack([b for _, b in pr]), device=dev)
    Xs4 = [torch.tensor(synthetic.sobol(1 << 20, 8, seed + 200 + q), device=dev) for q in range(P4)]
    bf4 = [float(b.max()) for _, b in pr]
    p = KernelParams("rbf", botorch_default_lengthscale(8), noise=1e-4)
    sts = eng.fit_batched(Xb, yb, p)
    lv = torch.empty((P4,), dtype=torch.float64, device=dev)
    li = torch.empty((P4,), dtype=torch.int64, device=dev)

    def share_step():
        ss = eng.fit_batched(Xb, yb, p, check=False, out=sts)
        eng.inverse_batched(ss)
        for q in range(P4):
            v, i = eng.acquire(ss[q], Xs4[q], "logei", best_f=bf4[q], index_offset=q << 20)
            lv[q:q + 1].copy_(v)
            li[q:q + 1].copy_(i)
        return eng.argmax_combine(lv, li)

    share_step()
    tf, ts = [], []
    for _ in range(5):
        torch.cuda.synchronize()
        a = time.perf_counter()
        eng.fit_batched(Xb, yb, p, check=False, out=sts)
        torch.cuda.synchronize()
        tf.append(time.perf_counter() - a)
    for _ in range(2):
        torch.cuda.synchronize()
        a = time.perf_counter()
        bv, bi = share_step()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - a)
    if any(st.pivot_failure() >= 0 for st in sts):
        raise RuntimeError("configs[3] share: Cholesky failed")
    f, t = float(np.median(tf)), float(np.median(ts))
    out["configs[3] per-GPU share"] = {
        "workload": "4 independent n=4096 d=8 RBF fp64 problems per GPU (32 restarts / 8 GPUs), batched posterior "
                    "update (batched_fit_ms), then batched L^-T + a 1048576-candidate logEI sweep each + argmax "
                    "combine (ms_per_step)",
        "problems": P4, "batched_fit_ms": 1e3 * f, "updates_per_s": P4 / f, "ms_per_step": 1e3 * t,
        "acq_cands_per_s": P4 * (1 << 20) / t, "best_index": int(bi.item())}
    del sts, Xb, yb, Xs4
    torch.cuda.empty_cache()
    # the driven variant (Bayesian7) at its own configuration: T = 8 tasks, M = 2048 inducing points
    # (random-init variational state of that shape), d = 5; a 10,000-candidate pool scan (score -> top 8000 -> FPS of
    # 500, optimization/Bayesian7.py:646-688) and the predictive's scoring rate on 2^20 candidates
    from bayesianoptimizer_amd.svgp import SVGPModel, SVGPPredictor
    rng = np.random.default_rng(seed + 19)
    T8, M8, d5 = 8, 2048, 5
    Z = rng.standard_normal((T8, M8, d5))
    vchol = np.tril(0.3 * rng.standard_normal((T8, M8, M8)) / np.sqrt(M8))
    for t in range(T8):
        vchol[t][np.diag_indices(M8)] = 0.2 + 0.5 * rng.random(M8)
    kps = [KernelParams("scale_linear_matern52", list(0.8 + rng.random(d5)), outputscale=0.5 + rng.random(),
                        noise=1e-3, const_mean=0.0, linear_variance=list(0.05 + 0.1 * rng.random(d5)))
           for _ in range(T8)]
    model = SVGPModel(Z=torch.tensor(Z), vmean=torch.tensor(rng.standard_normal((T8, M8))),
                      vchol=torch.tensor(vchol), params=kps)
    torch.cuda.synchronize()
    a = time.perf_counter()
    pred = SVGPPredictor(model, eng)
    torch.cuda.synchronize()
    t_prep = time.perf_counter() - a
    pool = torch.tensor(rng.random((10000, d5)), device=dev)
    big = torch.tensor(rng.random((1 << 20, d5)), device=dev)
    pred.pool_scan(pool, batch_k=500, start=0)
    pred.uncertainty(big, transformed=True)
    tp, tb = [], []
    for _ in range(3):
        torch.cuda.synchronize()
        a = time.perf_counter()
        pred.pool_scan(pool, batch_k=500, start=0)
        torch.cuda.synchronize()
        b = time.perf_counter()
        pred.uncertainty(big, transformed=True)
        torch.cuda.synchronize()
        tp.append(b - a)
        tb.append(time.perf_counter() - b)
    out["svgp driven config (Bayesian7)"] = {
        "workload": "batched SVGP predictive, T=8 tasks, M=2048 inducing points, d=5 (ScaleKernel(Linear+Matern-5/2) "
                    "per task): 10,000-candidate pool scan (variance-sum score, top 8000, FPS of 500) and the "
                    "score of 1048576 candidates",
        "prepare_ms": 1e3 * t_prep, "pool_scan_ms": 1e3 * float(np.median(tp)),
        "score_cands_per_s": (1 << 20) / float(np.median(tb)),
        "score_tflops_3M2_per_cand_task": 3.0 * M8 * M8 * T8 * (1 << 20) / float(np.median(tb)) / 1e12}
    del pred, model, pool, big
    torch.cuda.empty_cache()
    # the BO loop's per-iteration update done incrementally: one new observation appended to an
    # n = 4096 fit by the bordered Cholesky (gpx_append_f64; the same factor a refit computes, GPU parity tests),
    # beside the headline's full refit
    X_np, y_np = synthetic.problem(4097, 8, seed + 17)
    X, y = torch.tensor(X_np, device=dev), torch.tensor(y_np, device=dev)
    p = KernelParams("rbf", botorch_default_lengthscale(8), noise=1e-4)
    base = eng.fit(X[:4096], y[:4096], p, capacity=4224)
    ta = []
    for _ in range(7):
        base.n, base.npad = 4096, eng.padded_n(4096)
        torch.cuda.synchronize()
        a = time.perf_counter()
        st = eng.append(base, X, y, check=False)
        torch.cuda.synchronize()
        ta.append(time.perf_counter() - a)
    if st.pivot_failure() >= 0:
        raise RuntimeError("append Cholesky failed")
    t = float(np.median(ta))
    out["incremental n=4096+1"] = {"workload": "append 1 observation to an n=4096 d=8 RBF fit (bordered Cholesky, "
                                               "L^-T and alpha updated), exact", "update_ms": 1e3 * t,
                                   "updates_per_s": 1.0 / t}
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        rc = launch_ranks(args.gpus, argv)
        if args.launcher_selftest:
            print(json.dumps({"launcher": {"gpus": args.gpus, "rc": rc,
                                           "parent_hip_initialized": bool(torch.cuda.is_initialized())}}))
        sys.exit(rc)
    check_world(args)
    if args.launcher_selftest:
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                          "world_size": int(os.environ.get("WORLD_SIZE", "1")),
                          "hip_initialized": bool(torch.cuda.is_initialized())}), flush=True)
        return
    dist, rank, world, local = dist_setup(args)
    dev = torch.device("cuda", local)
    P = args.problems_per_gpu
    ls = botorch_default_lengthscale(args.d)
    params = KernelParams(args.kernel, ls, noise=1e-4)
    eng = GPEngine(dev)
    probs = []  # (X, y, Xs, best_f, global unit index)
    for q in range(P):
        unit = rank * P + q
        seed = args.seed + 1000 * unit
        X_np, y_np = synthetic.problem(args.n, args.d, seed)
        Xs_np = synthetic.sobol(args.m, args.d, seed + 1)
        X, y = torch.tensor(X_np, device=dev), torch.tensor(y_np, device=dev)
        Xs = torch.tensor(Xs_np, device=dev)
        probs.append((X, y, Xs, float(y_np.max()), unit))
    # P problems of one GPU are fitted together in the same launches (gpx_fit_batched_f64, BASELINE configs[3])
    Xb = torch.stack([p[0] for p in probs])
    yb = torch.stack([p[1] for p in probs])
    states = eng.fit_batched(Xb, yb, params) if P > 1 else [eng.fit(Xb[0], yb[0], params)]  # allocation outside
    X_np, y_np = synthetic.problem(args.n, args.d, args.seed + 1000 * rank * P)  # cpu-baseline inputs
    Xs_np = synthetic.sobol(args.m, args.d, args.seed + 1000 * rank * P + 1)

    def fit_all():
        if P > 1:
            return eng.fit_batched(Xb, yb, params, check=False, out=states)
        return [eng.fit(Xb[0], yb[0], params, check=False, out=states[0])]

    # the cross-rank exchange through libgpx's own RCCL communicator (gpx_allreduce_argmax): one 16-byte record per
    # rank, one all-gather, the deterministic combine kernel - no torch collective inside the timed step
    exchange = RCCLArgmaxExchange(eng) if dist is not None else None
    loc_v = torch.empty((P,), dtype=torch.float64, device=dev)
    loc_i = torch.empty((P,), dtype=torch.int64, device=dev)

    def step():
        sts = fit_all()
        if P > 1:
            eng.inverse_batched(sts)  # W = L^-T of every problem for its sweep, in the same launches
        for q, (Xq, yq, Xsq, bfq, unit) in enumerate(probs):
            bv, bi = eng.acquire(sts[q], Xsq, args.acq, best_f=bfq, index_offset=unit * args.m)
            loc_v[q:q + 1].copy_(bv)
            loc_i[q:q + 1].copy_(bi)
        bv, bi = eng.argmax_combine(loc_v, loc_i) if P > 1 else (loc_v[:1], loc_i[:1])
        if exchange is not None:
            bv, bi = exchange(bv, bi)
        return bv, bi

    for _ in range(args.warmup):
        step()
    barrier(dist)
    eng.timing_reset()
    eng.timing_enable(["trmm", "kstar"])
    t0 = time.perf_counter()
    for _ in range(args.steps):
        bv, bi = step()
    barrier(dist)
    elapsed = time.perf_counter() - t0
    trmm_ms, trmm_launches = eng.timing_query("trmm")
    kstar_ms, kstar_launches = eng.timing_query("kstar")
    eng.timing_disable()
    if any(st.pivot_failure() >= 0 for st in states):
        raise RuntimeError("Cholesky failed inside the benchmark")

    # fit-only loop: posterior updates per second (all P problems of a GPU per fit call)
    fit_reps = max(args.steps, 10)
    barrier(dist)
    t2 = time.perf_counter()
    for _ in range(fit_reps):
        fit_all()
    barrier(dist)
    fit_elapsed = time.perf_counter() - t2
    # per-kernel split of the update (hipEvents around each family, a separate loop so the timed one is event-free)
    eng.timing_reset()
    eng.timing_enable(["gram", "potrf", "alpha"])
    for _ in range(fit_reps):
        fit_all()
    part = {k: eng.timing_query(k) for k in ("gram", "potrf", "alpha")}
    eng.timing_disable()

    # latency of the cross-GPU exchange alone (report it separately; xGMI bandwidth is irrelevant for a
    # 16-byte record): back-to-back gpx_allreduce_argmax calls on the step's records, outside the timed step loop
    xch_us = None
    if exchange is not None:
        try:
            xr = 50
            barrier(dist)
            t3 = time.perf_counter()
            for _ in range(xr):
                exchange(bv.clone(), bi.clone())
            torch.cuda.synchronize()
            xch_us = 1e6 * (time.perf_counter() - t3) / xr
        except Exception as e:  # a measurement only: never fail the bench line over it
            print(f"exchange latency not measured: {e}", file=sys.stderr)
            xch_us = None

    times = torch.tensor([elapsed, fit_elapsed, xch_us if xch_us is not None else -1.0], dtype=torch.float64,
                         device=dev)
    if dist is not None:
        dist.all_reduce(times, op=dist.ReduceOp.MAX)
    elapsed, fit_elapsed = float(times[0]), float(times[1])
    xch_us = float(times[2]) if float(times[2]) >= 0 else None

    if rank == 0:
        m, n = args.m, args.n
        value = world * P * m * args.steps / elapsed
        avg_ms = trmm_ms / max(trmm_launches, 1)
        cands_per_launch = P * m * args.steps / max(trmm_launches, 1)
        flops_per_launch = float(n) * n * cands_per_launch  # n^2 flops per candidate (v = L^-1 k*)
        achieved = flops_per_launch / (avg_ms * 1e-3) / 1e12
        # kernel build K(X, X*): writes npad x C fp64 per launch, reads X and the chunk's candidates once
        npad = -(-n // 128) * 128
        kc = P * m * args.steps / max(kstar_launches, 1)
        kstar_bytes = 8.0 * (npad * kc + (n + kc) * args.d)
        kstar_avg = kstar_ms / max(kstar_launches, 1)
        kstar_gbs = kstar_bytes / (kstar_avg * 1e-3) / 1e9
        gram_bytes = P * 8.0 * (npad * (npad + 1) / 2 + n * args.d)
        gram_avg = part["gram"][0] / max(part["gram"][1], 1)
        gram_gbs = gram_bytes / (gram_avg * 1e-3) / 1e9
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(X_np, y_np, Xs_np, args.kernel, args.acq, ls, args.cpu_sample)
        extra = None
        if world == 1 and not args.no_other_configs:
            extra = other_configs(eng, dev, args.seed)
        traffic, traffic_src = pmc_traffic_record()
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "acq-cands/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded U[0,1] X, sin-sum y, scrambled Sobol candidates; fixed hyperparameters)",
            "config": {
                "workload": (f"BASELINE configs[1]: n={n} d={args.d} {args.kernel.upper()} GP fp64, one posterior "
                         f"update + {m}-candidate {args.acq} sweep + argmax per step, per GPU") if P == 1 else
                        (f"BASELINE configs[3] shape: {P} independent n={n} d={args.d} {args.kernel.upper()} problems "
                         f"per GPU ({P * world} total), each a posterior update + {m}-candidate {args.acq} sweep"),
                "n": n, "d": args.d, "m": m, "kernel": args.kernel, "acq": args.acq,
                "parallelism": f"{world * P} independent problems ({P} per GPU), RCCL 16-byte argmax all-gather",
                "problems_per_gpu": P,
            },
            "updates_per_s": world * P * fit_reps / fit_elapsed,
            "fit_ms": 1e3 * fit_elapsed / fit_reps,
            "update_breakdown_ms": {"gram": part["gram"][0] / fit_reps, "potrf": part["potrf"][0] / fit_reps,
                                    "alpha_potrs": part["alpha"][0] / fit_reps},
            # posterior update (Gram + Cholesky + alpha by triangular solves; the L^-T a sweep needs is built by the
            # sweep) against the fp64 MFMA roofline at SURVEY §8d's n^3/3 flops: a latency-bound chain of n/64
            # dependent panel launches, far from the bound
            "updates_roofline": {"flops_per_update": n ** 3 / 3.0,
                                 "achieved": (n ** 3 / 3.0) * P / (fit_elapsed / fit_reps) / 1e12,
                                 "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                                 "frac": (n ** 3 / 3.0) * P / (fit_elapsed / fit_reps) / 1e12 / FP64_PEAK_TFLOPS},
            "best": {"value": float(bv.item()), "index": int(bi.item())},
            "roofline": {
                "kernel": "trmm_sumsq_kernel (V = L^-1 K*, fp64 MFMA 16x16x4)",
                "bound": "mfma",
                "achieved": achieved,
                "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved / FP64_PEAK_TFLOPS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "avg_launch_ms": avg_ms,
                "launches": trmm_launches,
                "flops_per_launch": flops_per_launch,
            },
            # the kernel build against the HBM roofline (north star): its write of K* is the algorithmic traffic;
            # the fp64 exp per element keeps it VALU-bound below the HBM bound
            "kernel_build_roofline": {"kernel": "kstar_kernel (K(X, X*) for one candidate chunk)", "bound": "hbm",
                                      "achieved": kstar_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                      "frac": kstar_gbs / HBM_PEAK_GBS, "bytes_per_launch": kstar_bytes,
                                      "avg_launch_ms": kstar_avg, "launches": kstar_launches},
            # the training-set kernel build (gram_kernel) against HBM, as the north star asks: its algorithmic traffic
            # is the write of the lower triangle of the padded K, 8 npad (npad + 1) / 2 bytes (+ X read once)
            "gram_roofline": {"kernel": "gram_kernel (K(X, X) + noise I, lower triangle)", "bound": "hbm",
                              "achieved": gram_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": gram_gbs / HBM_PEAK_GBS, "bytes_per_launch": gram_bytes,
                              "avg_launch_ms": gram_avg, "launches": part["gram"][1]},
            "cpu_baseline": cpu,
            "exchange": {"collective": "RCCL all-gather of one 16-byte (value, index) record per rank + combine "
                                       "kernel (gpx_allreduce_argmax), max over ranks", "latency_us": xch_us}
            if world > 1 else None,
            "other_configs": extra,
        }
        print(json.dumps(out))
    if exchange is not None:
        exchange.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
