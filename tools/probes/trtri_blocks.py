"""Locate wrong blocks of W = L^{-T} (diagnostic): fit, inverse, then max |triu(W)^T L - I| per 128 x 128 block."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bayesianoptimizer_amd import GPEngine, KernelParams, botorch_default_lengthscale, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
dev = torch.device("cuda", 0)
X, y = synthetic.problem(n, 8, 1)
eng = GPEngine(dev)
p = KernelParams("matern52", botorch_default_lengthscale(8), noise=1e-4)
st = eng.fit(torch.tensor(X, device=dev), torch.tensor(y, device=dev), p)
eng.inverse(st)
L = torch.tril(st.L[:n, :n])
W = torch.triu(st.W[:n, :n])
E = W.T @ L
E -= torch.eye(n, device=dev, dtype=E.dtype)
nb = n // 128
B = E.abs().reshape(nb, 128, nb, 128).amax(dim=(1, 3)).cpu().numpy()
bad = np.argwhere(B > 1e-9)
print(f"n={n} max err {B.max():.3e}, {len(bad)} bad 128-blocks of {nb * nb}")
for r, c in bad[:40]:
    print(f"  block ({r},{c}) err {B[r, c]:.3e}")
# W itself: which 128-blocks of triu(W) differ from W of the transposed-solve definition W^T = L^{-1}
print("TRTRI BLOCKS DONE")
