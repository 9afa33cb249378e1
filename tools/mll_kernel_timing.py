"""MLL value + gradient kernel time (libgpx 'mll' launch timer) per covariance kind and n, d = 8."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bayesianoptimizer_amd import GPEngine, KernelParams, synthetic

eng = GPEngine(0)
dev = torch.device("cuda", 0)
for n in [int(a) for a in sys.argv[1:]] or [1024, 4096, 16384]:
    X, y = synthetic.problem(n, 8, 3)
    Xt, Yt = torch.tensor(X, device=dev), torch.tensor(y, device=dev).unsqueeze(-1)
    for kind in ("rbf", "matern52", "scale_linear_matern52"):
        p = KernelParams(kind, 0.5, noise=1e-3, linear_variance=0.2)
        st = eng.fit(Xt, Yt, p)
        eng.mll_grad(st, Yt)
        torch.cuda.synchronize()
        eng.timing_reset()
        eng.timing_enable(["mll"])
        for _ in range(5):
            g = eng.mll_grad(st, Yt)
        torch.cuda.synchronize()
        ms, _ = eng.timing_query("mll")
        eng.timing_disable()
        print(f"n={n} {kind}: mll value+grad {ms / 5:.3f} ms  (nll {float(g[0]):.6f})", flush=True)
print("MLL TIMING DONE")
