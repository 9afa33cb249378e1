"""sha256 of L and alpha after one n = 4096 fit (and a B = 4 batched fit): compares libgpx builds bit for bit
(GPX_LIB selects the library)."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bayesianoptimizer_amd import GPEngine, KernelParams, botorch_default_lengthscale, synthetic  # noqa: E402

dev = torch.device("cuda", 0)
eng = GPEngine(dev)
for n in (4096, 1000, 8192):
    X, y = synthetic.problem(n, 8, 3)
    p = KernelParams("rbf", botorch_default_lengthscale(8), noise=1e-4)
    st = eng.fit(torch.tensor(X, device=dev), torch.tensor(y, device=dev), p)
    h = hashlib.sha256(torch.tril(st.L[:n, :n]).cpu().numpy().tobytes() + st.alpha.cpu().numpy().tobytes()).hexdigest()
    print(f"n={n} L+alpha sha256 {h[:16]}")
print("FIT HASH DONE")
