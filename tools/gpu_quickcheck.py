"""Quick GPU sanity run of every engine stage against the oracle (diagnostic script, not a test)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from bayesianoptimizer_amd import GPEngine, KernelParams
from oracle import gp_oracle as O

def run(n, d, kind, m, nrhs=1, seed=0):
    X, y = O.synthetic_problem(n, d, seed)
    Y = np.stack([y * (r + 1) for r in range(nrhs)], 1)
    ls = O.botorch_default_lengthscale(d)
    kp = KernelParams(kind=kind, lengthscale=ls, noise=1e-4, linear_variance=0.3)
    op = O.KernelParams(kind={"rbf":0,"matern52":1,"scale_linear_matern52":2}[kind], lengthscale=np.full(d, ls), noise=1e-4, linear_variance=np.full(d,0.3))
    eng = GPEngine(0)
    Xt = torch.tensor(X, device="cuda"); Yt = torch.tensor(Y, device="cuda")
    K = eng.gram(Xt, kp); Kref = O.gram(X, op)
    Kg = torch.tril(K).cpu().numpy()[:n,:n]
    print(f"[n={n} d={d} {kind}] gram max|dK| lower = {np.abs(np.tril(Kref)-Kg).max():.3e}")
    st = eng.fit(Xt, Yt, kp)
    torch.cuda.synchronize()
    L = torch.tril(st.L).cpu().numpy()[:n,:n]
    Lref = O.cholesky(Kref)
    print(f"  chol max|dL| = {np.abs(L-Lref).max():.3e}  info={int(st.info.item())}")
    eng.inverse(st)  # a factor-only update leaves W unbuilt (GPState.W_ready False); build it before reading
    W = st.W.cpu().numpy()
    Winv_ref = np.linalg.inv(Lref).T
    print(f"  W max|dW| (upper) = {np.abs(np.triu(W[:n,:n]) - Winv_ref).max():.3e}, max|W|={np.abs(Winv_ref).max():.3e}")
    ost = O.fit(X, Y, op)
    a = st.alpha.cpu().numpy()[:n]
    print(f"  alpha rel err = {np.abs(a-ost.alpha.reshape(n,-1)).max()/np.abs(ost.alpha).max():.3e}")
    Xs = O.sobol_candidates(m, d, seed+1)
    mu, var = eng.posterior(st, torch.tensor(Xs, device="cuda"))
    mu_r, var_r = O.posterior(ost, Xs)
    mu_g = mu.cpu().numpy(); var_g = var.cpu().numpy()
    print(f"  posterior |dmu|/max|mu| = {np.abs(mu_g[:,0]-(mu_r if mu_r.ndim==1 else mu_r[:,0])).max()/np.abs(mu_r).max():.3e}  |dvar| = {np.abs(var_g-var_r).max():.3e}")
    best_f = float(y.max())
    for acq, kid in (("logei",1),("ei",0),("ucb",2),("variance",3)):
        o1 = O.fit(X, Y[:,0], op)
        vref, iref, sref = O.acquire_argmax(o1, Xs, kid, best_f=best_f, beta=4.0)
        bv, bi, sc = eng.acquire(st, torch.tensor(Xs, device="cuda"), acq, best_f=best_f, beta=4.0, return_scores=True)
        scg = sc.cpu().numpy()
        fin = np.isfinite(sref)
        print(f"  {acq}: gpu ({bv.item():.12g},{bi.item()}) ref ({vref:.12g},{iref}) max|dscore|={np.abs(scg[fin]-sref[fin]).max():.3e}")

def timeit(n, d, m):
    X, y = O.synthetic_problem(n, d, 0)
    kp = KernelParams(kind="rbf", lengthscale=O.botorch_default_lengthscale(d), noise=1e-4)
    eng = GPEngine(0)
    Xt = torch.tensor(X, device="cuda"); Yt = torch.tensor(y, device="cuda")
    st = eng.fit(Xt, Yt, kp)
    Xs = torch.tensor(O.sobol_candidates(m, d, 1), device="cuda")
    eng.acquire(st, Xs, "logei", best_f=float(y.max()))
    torch.cuda.synchronize()
    eng.timing_enable(["gram","potrf","trtri","alpha","kstar","trmm","acq"])
    for rep in range(3):
        eng.timing_reset()
        t0=time.perf_counter(); st = eng.fit(Xt, Yt, kp, check=False, out=st); torch.cuda.synchronize(); t1=time.perf_counter()
        bv, bi = eng.acquire(st, Xs, "logei", best_f=float(y.max())); torch.cuda.synchronize(); t2=time.perf_counter()
        parts = {k: eng.timing_query(k) for k in ["gram","potrf","trtri","alpha","kstar","trmm","acq"]}
        print(f"[time n={n} m={m}] fit {1e3*(t1-t0):.2f} ms, sweep {1e3*(t2-t1):.2f} ms; " + ", ".join(f"{k}={v[0]:.3f}ms/{v[1]}" for k,v in parts.items()))
    tr = parts["trmm"]
    fl = float(n)*n*m
    print(f"  trmm achieved {fl/(tr[0]*1e-3)/1e12:.2f} TF/s (algorithmic n^2 m)")

if __name__ == "__main__":
    run(300, 4, "rbf", 1000)
    run(200, 5, "scale_linear_matern52", 777, nrhs=3)
    run(1000, 8, "matern52", 5000)
    run(4096, 8, "rbf", 20000)
    timeit(4096, 8, 1 << 20)
