"""Leading-dimension padding of the factor / inverse buffers (diagnostic): the fit (Gram + Cholesky + backward solve) and
W = L^-T with L and W allocated as npad x (npad + pad) buffers (row stride npad + pad doubles) against the default
npad x npad (a power-of-two row stride at n = 4096 / 8192 / 16384), alternating, median of rounds; alpha compared.

  python tools/ld_pad_ab.py --n 16384 --kernel matern52 --pads 0 16 64
"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bayesianoptimizer_amd import GPEngine, KernelParams, botorch_default_lengthscale, synthetic  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=16384)
ap.add_argument("--d", type=int, default=8)
ap.add_argument("--kernel", default="matern52")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--pads", type=int, nargs="+", default=[0, 16, 64])
a = ap.parse_args()
X, y = synthetic.problem(a.n, a.d, 0)
dev = torch.device("cuda", 0)
eng = GPEngine(dev)
p = KernelParams(a.kernel, botorch_default_lengthscale(a.d), noise=1e-4)
Xt, yt = torch.tensor(X, device=dev), torch.tensor(y, device=dev)
npad = eng.padded_n(a.n)
states = {}
for pad in a.pads:
    st = eng.alloc_state(Xt, 1, p)
    if pad:
        st.L = torch.empty((npad, npad + pad), dtype=torch.float64, device=dev)[:, :npad]
        st.W = torch.empty((npad, npad + pad), dtype=torch.float64, device=dev)[:, :npad]
    states[pad] = st
fit_t = {pad: [] for pad in a.pads}
inv_t = {pad: [] for pad in a.pads}
alpha0 = None
for rnd in range(a.rounds):
    for pad in a.pads:
        st = eng.fit(Xt, yt, p, out=states[pad])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            st = eng.fit(Xt, yt, p, check=False, out=st)
        torch.cuda.synchronize()
        fit_t[pad].append((time.perf_counter() - t0) / a.reps * 1e3)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            st.W_ready = False
            eng.inverse(st)
        torch.cuda.synchronize()
        inv_t[pad].append((time.perf_counter() - t0) / a.reps * 1e3)
        if rnd == 0:
            al = st.alpha.clone()
            if alpha0 is None:
                alpha0 = al
            print(f"pad {pad}: ld {st.L.stride(0)}, alpha bitwise equal to pad {a.pads[0]}: {bool(torch.equal(al, alpha0))}",
                  flush=True)
for pad in a.pads:
    print(f"n={a.n} {a.kernel} pad {pad:3d}: fit {statistics.median(fit_t[pad]):.3f} ms  inverse "
          f"{statistics.median(inv_t[pad]):.3f} ms")
print("LD PAD AB DONE")
