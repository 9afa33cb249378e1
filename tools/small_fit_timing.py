"""Small-n posterior-update latency: wall time of GPEngine.fit (check=False, buffers reused) against the sum of
libgpx's GPU phase timers, and the same fit replayed from a HIP graph (torch.cuda.CUDAGraph capture of the libgpx
launches on torch's current stream).  Shows whether the update at the reference's own sizes is host-launch-bound."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from bayesianoptimizer_amd import GPEngine, KernelParams, botorch_default_lengthscale, synthetic

dev = torch.device("cuda", 0)
eng = GPEngine(dev)


def med(fn, reps=50):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        a = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - a)
    ts.sort()
    return 1e3 * ts[len(ts) // 2]


for n in [int(a) for a in sys.argv[1:]] or [64, 128, 256, 512, 1024, 4096]:
    d = 8
    X, y = synthetic.problem(n, d, 3)
    X, y = torch.tensor(X, device=dev), torch.tensor(y, device=dev)
    p = KernelParams("rbf", botorch_default_lengthscale(d), noise=1e-4)
    st = eng.fit(X, y, p)
    wall = med(lambda: eng.fit(X, y, p, check=False, out=st))
    eng.timing_reset()
    eng.timing_enable(["gram", "potrf", "trtri", "alpha"])
    reps = 20
    for _ in range(reps):
        eng.fit(X, y, p, check=False, out=st)
    torch.cuda.synchronize()
    ph = {k: eng.timing_query(k)[0] / reps for k in ("gram", "potrf", "trtri", "alpha")}
    eng.timing_disable()
    L_ref = st.L.clone()
    line = (f"n={n}: fit wall {wall:.3f} ms; GPU phases gram {ph['gram']:.3f} potrf {ph['potrf']:.3f} "
            f"trtri {ph['trtri']:.3f} alpha {ph['alpha']:.3f} (sum {sum(ph.values()):.3f} ms)")
    try:
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            eng.fit(X, y, p, check=False, out=st)  # warm the workspace on the capture stream
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            eng.fit(X, y, p, check=False, out=st)
        torch.cuda.synchronize()
        st.L.zero_()
        g.replay()
        torch.cuda.synchronize()
        same = bool(torch.equal(torch.tril(st.L[:n, :n]), torch.tril(L_ref[:n, :n])))
        gt = med(g.replay)
        line += f"; graph replay {gt:.3f} ms (L identical: {same})"
    except Exception as e:  # noqa: BLE001
        line += f"; graph capture failed: {type(e).__name__}: {e}"
    print(line, flush=True)
print("SMALL FIT DONE")
