"""Flush interval A/B of the multi-launch Cholesky at one n (handle options potrf_mode / potrf_lazy), alternating."""
import argparse, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bayesianoptimizer_amd import GPEngine, KernelParams, botorch_default_lengthscale, synthetic

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=16384)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--plans", default="1:8,1:4,1:6,1:12")
a = ap.parse_args()
dev = torch.device("cuda", 0)
eng = GPEngine(dev)
p = KernelParams("matern52", botorch_default_lengthscale(8), noise=1e-4)
X, y = synthetic.problem(a.n, 8, 0)
Xt, yt = torch.tensor(X, device=dev), torch.tensor(y, device=dev)
st = eng.fit(Xt, yt, p)
eng.timing_enable(["potrf"])
for rnd in range(2):
    for plan in a.plans.split(","):
        mode, g = (int(v) for v in plan.split(":"))
        eng.set_option("potrf_mode", mode)
        eng.set_option("potrf_lazy", g)
        st = eng.fit(Xt, yt, p, check=True, out=st)
        torch.cuda.synchronize()
        eng.timing_reset()
        for _ in range(a.reps):
            st = eng.fit(Xt, yt, p, check=False, out=st)
        torch.cuda.synchronize()
        ms, cnt = eng.timing_query("potrf")
        print(f"round {rnd} n={a.n} mode {mode} g {g}: potrf {ms / cnt:.3f} ms", flush=True)
