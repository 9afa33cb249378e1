"""Diagnostic: where a batched inverse-path fit on an uncached factor differs from its single fit (GPX_UNCACHED_FACTOR=1).
Prints, per problem, the 64x64 blocks of L (lower triangle) whose bits differ, and whether W / alpha differ."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from bayesianoptimizer_amd import GPEngine, KernelParams
from oracle import gp_oracle as O

n, B, d = int(sys.argv[1]) if len(sys.argv) > 1 else 300, 3, 6
inverse = (sys.argv[2] != "0") if len(sys.argv) > 2 else True
e = GPEngine(0)
dev = torch.device("cuda", 0)
kp = KernelParams("matern52", O.botorch_default_lengthscale(d), noise=2e-4)
Xs, Ys = [], []
for b in range(B):
    X, y = O.synthetic_problem(n, d, 100 + b)
    Xs.append(X)
    Ys.append(y[:, None])
t = lambda a: torch.tensor(a, device=dev)
sts = e.fit_batched(t(np.stack(Xs)), t(np.stack(Ys)), kp, inverse=inverse)
for b in range(B):
    s = e.fit(t(Xs[b]), t(Ys[b]), kp, inverse=inverse)
    La, Lb = torch.tril(sts[b].L[:n, :n]).cpu().numpy(), torch.tril(s.L[:n, :n]).cpu().numpy()
    diff = La != Lb
    blocks = sorted({(i // 64, j // 64) for i, j in zip(*np.nonzero(diff))})
    print(f"problem {b}: {int(diff.sum())} differing L entries, blocks {blocks[:12]}, max |dL| {np.abs(La - Lb).max():.3e}, "
          f"alpha equal {torch.equal(sts[b].alpha, s.alpha)}")
