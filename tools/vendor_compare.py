"""Vendor-library context for the posterior update: torch.linalg (rocSOLVER / hipBLAS) fp64 Cholesky, triangular
inverse and the sweep product on the same MI355X, beside libgpx's own kernels (timed with libgpx's hipEvent timers).
Context only: the product path never calls these.  usage: python tools/vendor_compare.py [n ...]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bayesianoptimizer_amd import GPEngine, KernelParams, botorch_default_lengthscale, synthetic

dev = torch.device("cuda", 0)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - a)
    ts.sort()
    return 1e3 * ts[len(ts) // 2]


eng = GPEngine(0)
for n in [int(a) for a in sys.argv[1:]] or [1024, 4096, 8192, 16384]:
    X, y = synthetic.problem(n, 8, 3)
    p = KernelParams("rbf", botorch_default_lengthscale(8), noise=1e-4)
    Xt, yt = torch.tensor(X, device=dev), torch.tensor(y, device=dev)
    st = eng.fit(Xt, yt, p)
    ls = botorch_default_lengthscale(8)
    K = torch.exp(-0.5 * torch.cdist(Xt / ls, Xt / ls).square()) + 1e-4 * torch.eye(n, device=dev, dtype=torch.float64)
    t_chol = timed(lambda: torch.linalg.cholesky(K))
    L = torch.linalg.cholesky(K)
    I = torch.eye(n, device=dev, dtype=torch.float64)
    t_inv = timed(lambda: torch.linalg.solve_triangular(L, I, upper=False))
    Ks = torch.rand(n, 8192, device=dev, dtype=torch.float64)
    t_trsm = timed(lambda: torch.linalg.solve_triangular(L, Ks, upper=False))
    Winv = torch.linalg.solve_triangular(L, I, upper=False)
    t_gemm = timed(lambda: Winv @ Ks)
    eng.timing_reset()
    eng.timing_enable(["gram", "potrf", "trtri", "alpha"])
    t_fit = timed(lambda: eng.fit(Xt, yt, p, check=False, out=st))
    r = {k: eng.timing_query(k) for k in ("potrf", "trtri")}
    eng.timing_disable()
    reps = 6  # fits inside timed(): one warm-up + 5
    fl = n ** 3 / 3
    print(f"n={n}: rocSOLVER potrf {t_chol:.3f} ms ({fl / t_chol / 1e9:.1f} TF/s) | libgpx potrf "
          f"{r['potrf'][0] / reps:.3f} ms ({fl / (r['potrf'][0] / reps) / 1e9:.1f} TF/s); "
          f"L^-1 by torch trsm {t_inv:.3f} ms vs libgpx trtri {r['trtri'][0] / reps:.3f} ms; "
          f"libgpx full update {t_fit:.3f} ms; torch trsm L^-1 K* (8192 cands) {t_trsm:.3f} ms "
          f"({n * n * 8192 / t_trsm / 1e9:.1f} TF/s), torch dgemm L^-1 K* {t_gemm:.3f} ms "
          f"({2 * n * n * 8192 / t_gemm / 1e9:.1f} TF/s dense)", flush=True)
    del K, L, I, Ks, Winv, st
    torch.cuda.empty_cache()
print("VENDOR DONE")
