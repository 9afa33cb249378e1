"""A/B of the Cholesky schedules on one box: factor-only posterior updates (Gram + Cholesky + alpha by potrs) with
potrf_schedule = 1 (multi-launch) and 2 (dataflow), alternating, single and batched; live hipEvent split per part."""
import argparse, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bayesianoptimizer_amd import GPEngine, KernelParams, botorch_default_lengthscale, synthetic

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--d", type=int, default=8)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--batch", type=int, default=4)
ap.add_argument("--schedules", default="1,2")
a = ap.parse_args()
dev = torch.device("cuda", 0)
eng = GPEngine(dev)
p = KernelParams("rbf", botorch_default_lengthscale(a.d), noise=1e-4)
X, y = synthetic.problem(a.n, a.d, 0)
Xt, yt = torch.tensor(X, device=dev), torch.tensor(y, device=dev)
Xb = torch.stack([torch.tensor(synthetic.problem(a.n, a.d, s)[0], device=dev) for s in range(a.batch)])
yb = torch.stack([torch.tensor(synthetic.problem(a.n, a.d, s)[1], device=dev) for s in range(a.batch)])
scheds = [int(s) for s in a.schedules.split(",")]
st = eng.fit(Xt, yt, p)
stb = eng.fit_batched(Xb, yb, p)
ref = None
parts = ["gram", "potrf", "alpha"]
eng.timing_enable(parts)
for rnd in range(2):
    for s in scheds:
        eng.set_option("potrf_schedule", s)
        st = eng.fit(Xt, yt, p, check=True, out=st)
        a0 = st.alpha.clone()
        if ref is None:
            ref = a0
        diff = float((a0 - ref).abs().max())
        torch.cuda.synchronize()
        eng.timing_reset()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            st = eng.fit(Xt, yt, p, check=False, out=st)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.reps * 1e3
        split = {k: eng.timing_query(k)[0] / a.reps for k in parts}
        eng.timing_reset()
        t0 = time.perf_counter()
        for _ in range(max(1, a.reps // 4)):
            stb = eng.fit_batched(Xb, yb, p, check=False, out=stb)
        torch.cuda.synchronize()
        wb = (time.perf_counter() - t0) / max(1, a.reps // 4) * 1e3
        print(f"round {rnd} schedule {s}: update {wall:.3f} ms (" + ", ".join(f"{k} {v:.3f}" for k, v in split.items())
              + f"), batched x{a.batch} {wb:.3f} ms, max|dalpha| vs first {diff:.2e}", flush=True)
