"""Incremental update timing: gpx_append_f64 of q new points onto an n-point fit vs a full refit."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from bayesianoptimizer_amd import GPEngine, KernelParams, botorch_default_lengthscale, synthetic

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--d", type=int, default=8)
ap.add_argument("--q", default="1,64,256,512")
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda", 0)
eng = GPEngine(dev)
p = KernelParams("rbf", botorch_default_lengthscale(a.d), noise=1e-4)
qmax = max(int(v) for v in a.q.split(","))
X, y = synthetic.problem(a.n + qmax, a.d, 0)
Xt, yt = torch.tensor(X, device=dev), torch.tensor(y, device=dev)


def best(fn):
    ts = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return 1e3 * min(ts)


base = eng.fit(Xt[:a.n], yt[:a.n], p, capacity=a.n + qmax)
torch.cuda.synchronize()
for q in (int(v) for v in a.q.split(",")):
    n1 = a.n + q
    st_box = {}

    def do_append():
        # re-append onto the same base each rep: rows >= floor(n/128)*128 are rewritten, the kept block is untouched
        base.n, base.npad = a.n, eng.padded_n(a.n)
        st_box["s"] = eng.append(base, Xt[:n1], yt[:n1], check=False)

    t_app = best(do_append)
    ref = {}
    t_fit = best(lambda: ref.setdefault("s", eng.fit(Xt[:n1], yt[:n1], p, check=False)))
    s = st_box["s"]
    err = (torch.tril(s.L[:n1, :n1]) - torch.tril(eng.fit(Xt[:n1], yt[:n1], p).L[:n1, :n1])).abs().max().item()
    print(f"n={a.n} + q={q}: append {t_app:.3f} ms, refit {t_fit:.3f} ms ({t_fit / t_app:.1f}x); max|dL| {err:.2e}",
          flush=True)
