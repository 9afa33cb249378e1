"""Minimal driver for profiling the sweep kernels: one fit + `reps` logEI sweeps (n=4096 d=8, m candidates)."""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bayesianoptimizer_amd import GPEngine, KernelParams, botorch_default_lengthscale, synthetic

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--d", type=int, default=8)
ap.add_argument("--m", type=int, default=1 << 17)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--fit-only", action="store_true")
a = ap.parse_args()
X, y = synthetic.problem(a.n, a.d, 0)
Xs = synthetic.sobol(a.m, a.d, 1)
eng = GPEngine(0)
dev = torch.device("cuda", 0)
p = KernelParams("rbf", botorch_default_lengthscale(a.d), noise=1e-4)
Xt, yt, Xst = torch.tensor(X, device=dev), torch.tensor(y, device=dev), torch.tensor(Xs, device=dev)
st = eng.fit(Xt, yt, p)
for _ in range(a.reps):
    if a.fit_only:
        st = eng.fit(Xt, yt, p, check=False, out=st)
    else:
        bv, bi = eng.acquire(st, Xst, "logei", best_f=float(y.max()))
torch.cuda.synchronize()
print("done", float(bv.item()) if not a.fit_only else "")
