"""A/B timing of the Cholesky schedules (persistent dataflow vs multi-launch) at a given n, with a factor check:
both schedules must give the same L bit for bit (same arithmetic in the same order)."""
import argparse, os, subprocess, sys
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--child", default="")
a = ap.parse_args()
if not a.child:
    for mode in ("0", "1") if os.environ.get("AB_BOTH") else ("0",):
        env = dict(os.environ, GPX_POTRF_PERSIST=mode)
        r = subprocess.run([sys.executable, __file__, "--n", str(a.n), "--reps", str(a.reps), "--child", mode], env=env,
                           capture_output=True, text=True, timeout=300)
        sys.stdout.write(r.stdout)
        sys.stderr.write(r.stderr[-2000:])
        if r.returncode:
            sys.exit(r.returncode)
    sys.exit(0)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time
import numpy as np
import torch
from bayesianoptimizer_amd import GPEngine, KernelParams, botorch_default_lengthscale, synthetic
X, y = synthetic.problem(a.n, 8, 0)
dev = torch.device("cuda", 0)
eng = GPEngine(dev)
p = KernelParams("rbf", botorch_default_lengthscale(8), noise=1e-4)
Xt, yt = torch.tensor(X, device=dev), torch.tensor(y, device=dev)
st = eng.fit(Xt, yt, p)
torch.cuda.synchronize()
eng.timing_enable(["potrf", "alpha", "gram"])
best = 1e9
for r in range(a.reps):
    eng.timing_reset()
    st = eng.fit(Xt, yt, p, check=False, out=st)
    torch.cuda.synchronize()
    best = min(best, eng.timing_query("potrf")[0])
info = int(st.info.item())
L = torch.tril(st.L).cpu().numpy()
h = float(np.abs(L).sum())
np.save(f"/tmp/L_{a.child}.npy", L[:: max(1, a.n // 512), :])
same = ""
if a.child == "1" and os.path.exists("/tmp/L_0.npy"):
    L0 = np.load("/tmp/L_0.npy")
    same = f" identical_to_multilaunch={bool(np.array_equal(L0, L[:: max(1, a.n // 512), :]))}"
print(f"persist={a.child} n={a.n}: potrf best {best:.3f} ms, info={info}, sum|L|={h:.12e}{same}")
