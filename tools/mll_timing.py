"""End-to-end hyperparameter fit timing: ExactGP.fit_hyperparameters on the GPU engine at several
n, with the number of L-BFGS-B objective evaluations and the per-evaluation wall time (fit + MLL gradient + host)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from bayesianoptimizer_amd import GPEngine, KernelParams, synthetic
from bayesianoptimizer_amd.models import ExactGP

eng = GPEngine(torch.device("cuda", 0))
for n in [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "256,1024,4096").split(",")]:
    X, y = synthetic.problem(n, 8, 3)
    gp = ExactGP(X, y, KernelParams("rbf", 0.5, noise=1e-3), engine=eng)
    gp.fit_hyperparameters("dim_scaled")  # warm-up (allocations, code paths)
    gp = ExactGP(X, y, KernelParams("rbf", 0.5, noise=1e-3), engine=eng)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gp.fit_hyperparameters("dim_scaled")
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    r = gp.mll_result
    # GPU-only cost of one evaluation: fit + gradient, back to back
    st = gp.state
    Yt = torch.tensor(y, device=eng.device).unsqueeze(-1)
    torch.cuda.synchronize()
    a = time.perf_counter()
    for _ in range(10):
        st = eng.fit(gp.train_X, Yt, gp.params, check=False, out=st)
        eng.mll_grad(st, Yt)
    torch.cuda.synchronize()
    per = (time.perf_counter() - a) / 10
    print(f"n={n}: fit_hyperparameters {1e3 * dt:.1f} ms, {r.n_evals} evals ({1e3 * dt / max(r.n_evals, 1):.2f} ms "
          f"per eval); device fit+grad {1e3 * per:.2f} ms; nll {r.nll:.4f} success={r.success}", flush=True)
