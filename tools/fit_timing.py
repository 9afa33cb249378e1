"""Fit timing and factor-residual check at a given size (BASELINE configs[2]: n=16384 d=8 Matérn-5/2)."""
import argparse, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from bayesianoptimizer_amd import GPEngine, KernelParams, botorch_default_lengthscale, synthetic

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=16384)
ap.add_argument("--d", type=int, default=8)
ap.add_argument("--kernel", default="matern52")
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
X, y = synthetic.problem(a.n, a.d, 0)
dev = torch.device("cuda", 0)
eng = GPEngine(dev)
p = KernelParams(a.kernel, botorch_default_lengthscale(a.d), noise=1e-4)
Xt, yt = torch.tensor(X, device=dev), torch.tensor(y, device=dev)
st = eng.fit(Xt, yt, p)
torch.cuda.synchronize()
eng.timing_enable(["gram", "potrf", "trtri", "alpha"])
for inverse in (False, True):
    ts = []
    for r in range(a.reps):
        eng.timing_reset()
        t0 = time.perf_counter()
        st = eng.fit(Xt, yt, p, check=False, out=st, inverse=inverse)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
        parts = {k: eng.timing_query(k)[0] for k in ["gram", "potrf", "trtri", "alpha"]}
    what = "fit + L^-T (gpx_fit_f64)" if inverse else "update (gpx_fit_factor_f64: alpha by potrs)"
    print(f"n={a.n} {what}: {1e3*min(ts):.3f} ms (best of {a.reps}); " +
          ", ".join(f"{k} {v:.3f} ms" for k, v in parts.items()))
flops = a.n ** 3 / 3
print(f"  potrf {flops / (parts['potrf'] * 1e-3) / 1e12:.1f} TF/s, trtri {flops / (parts['trtri'] * 1e-3) / 1e12:.1f} TF/s (n^3/3 each)")
# residual on sampled rows: (L L^T)[rows] vs K[rows]
rows = np.sort(np.random.default_rng(0).choice(a.n, 32, replace=False))
L = torch.tril(st.L[:, :a.n])
Lr = L[torch.tensor(rows, device=dev)]
R = Lr @ L.T
from oracle import gp_oracle as O  # checker
op = O.KernelParams({"rbf": 0, "matern52": 1}[a.kernel], np.full(a.d, botorch_default_lengthscale(a.d)), noise=1e-4)
Kr = O.kernel_matrix(X[rows], X, op)
Kr[np.arange(32), rows] += 1e-4
print(f"  max |L L^T - K| on 32 rows: {np.abs(R.cpu().numpy() - Kr).max():.3e}; info={int(st.info.item())}")
# marginal-likelihood gradient kernel (K^{-1} = W W^T contraction, n^3/3 flops)
eng.timing_enable(["mll"])
eng.timing_reset()
for r in range(a.reps):
    g = eng.mll_grad(st, yt)
torch.cuda.synchronize()
ms, cnt = eng.timing_query("mll")
print(f"  mll grad: {ms / cnt:.3f} ms per call ({flops / (ms / cnt * 1e-3) / 1e12:.1f} TF/s n^3/3); nll={float(g[0]):.6f}")
