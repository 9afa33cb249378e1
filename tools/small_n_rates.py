"""Sweep rate across training-set sizes (the reference's own loops run n = 10^2..10^3): fit + 2^22-candidate logEI
sweep per n, candidates/s and the trmm share (libgpx launch timers)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bayesianoptimizer_amd import GPEngine, KernelParams, botorch_default_lengthscale, synthetic

dev = torch.device("cuda", 0)
eng = GPEngine(0)
m = 1 << 22
Xs = torch.tensor(synthetic.sobol(m, 8, 2), device=dev)
for n in [int(a) for a in sys.argv[1:]] or [64, 256, 1024, 2048]:
    X, y = synthetic.problem(n, 8, 1)
    p = KernelParams("rbf", botorch_default_lengthscale(8), noise=1e-4)
    st = eng.fit(torch.tensor(X, device=dev), torch.tensor(y, device=dev), p)
    bf = float(y.max())
    eng.acquire(st, Xs, "logei", best_f=bf)
    torch.cuda.synchronize()
    eng.timing_reset()
    eng.timing_enable(["kstar", "trmm", "acq"])
    a = time.perf_counter()
    for _ in range(3):
        eng.acquire(st, Xs, "logei", best_f=bf)
    torch.cuda.synchronize()
    t = (time.perf_counter() - a) / 3
    tm = {k: eng.timing_query(k)[0] / 3 for k in ("kstar", "trmm", "acq")}
    eng.timing_disable()
    print(f"n={n}: {m / t:.3e} candidates/s ({t * 1e3:.2f} ms per 2^22); kstar {tm['kstar']:.2f} ms, "
          f"trmm {tm['trmm']:.2f} ms ({n * n * m / (tm['trmm'] * 1e-3) / 1e12:.1f} TF/s), finalize {tm['acq']:.2f} ms",
          flush=True)
print("RATES DONE")
