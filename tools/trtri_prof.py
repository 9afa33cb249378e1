"""Triangular inverse W = L^{-T} at a large size (rocprofv3 target): one fit, then `reps` trtri calls on its factor.

  rocprofv3 --kernel-trace --stats -d gpurun_out/trtri -- python tools/trtri_prof.py --n 16384
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bayesianoptimizer_amd import GPEngine, KernelParams, botorch_default_lengthscale, synthetic  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=16384)
ap.add_argument("--d", type=int, default=8)
ap.add_argument("--kernel", default="matern52")
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
X, y = synthetic.problem(a.n, a.d, 0)
dev = torch.device("cuda", 0)
eng = GPEngine(dev)
p = KernelParams(a.kernel, botorch_default_lengthscale(a.d), noise=1e-4)
st = eng.fit(torch.tensor(X, device=dev), torch.tensor(y, device=dev), p)
torch.cuda.synchronize()
for _ in range(a.reps):
    t0 = time.perf_counter()
    W = eng.trtri(st.L, st.Dinv, a.n)
    torch.cuda.synchronize()
    print(f"n={a.n} trtri {1e3 * (time.perf_counter() - t0):.3f} ms", flush=True)
print("TRTRI PROF DONE")
