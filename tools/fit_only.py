"""A few factor-only posterior updates (Gram + Cholesky + potrs) at one size, for rocprofv3 counter passes."""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bayesianoptimizer_amd import GPEngine, KernelParams, botorch_default_lengthscale, synthetic
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--d", type=int, default=8)
ap.add_argument("--kernel", default="rbf")
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
X, y = synthetic.problem(a.n, a.d, 0)
dev = torch.device("cuda", 0)
eng = GPEngine(dev)
p = KernelParams(a.kernel, botorch_default_lengthscale(a.d), noise=1e-4)
Xt, yt = torch.tensor(X, device=dev), torch.tensor(y, device=dev)
st = eng.fit(Xt, yt, p)
for _ in range(a.reps):
    st = eng.fit(Xt, yt, p, check=False, out=st)
torch.cuda.synchronize()
print("fits done, info", int(st.info.item()))
