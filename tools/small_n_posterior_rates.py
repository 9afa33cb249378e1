"""Multi-output posterior rate at small n (Bayesian2.predict's 8 outputs sharing X): 2^22 candidates, d = 8."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from bayesianoptimizer_amd import GPEngine, KernelParams, botorch_default_lengthscale, synthetic

dev = torch.device("cuda", 0)
eng = GPEngine(0)
m, nrhs = 1 << 22, 8
Xs = torch.tensor(synthetic.sobol(m, 8, 2), device=dev)
for n in [int(a) for a in sys.argv[1:]] or [64, 128, 256]:
    X, y = synthetic.problem(n, 8, 1)
    Y = np.stack([y * (r + 1) for r in range(nrhs)], axis=1)
    p = KernelParams("rbf", botorch_default_lengthscale(8), noise=1e-4)
    st = eng.fit(torch.tensor(X, device=dev), torch.tensor(Y, device=dev), p)
    eng.posterior(st, Xs)
    torch.cuda.synchronize()
    a = time.perf_counter()
    for _ in range(3):
        eng.posterior(st, Xs)
    torch.cuda.synchronize()
    t = (time.perf_counter() - a) / 3
    print(f"n={n} outputs={nrhs}: {m / t:.3e} candidates/s ({t * 1e3:.2f} ms per 2^22)", flush=True)
print("POSTERIOR RATES DONE")
