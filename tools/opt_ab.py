"""A/B of handle options on the posterior update (gpx_fit_factor_f64) in ONE process: every arm is timed in alternating
rounds (median of the rounds), with the Gram / Cholesky / solve split from libgpx's own hipEvent timers, and the arm's
alpha compared bit for bit with the first arm's.

  python tools/opt_ab.py --n 4096 --arms "potrf_half=0" "potrf_half=-1" "potrf_half=1"
  python tools/opt_ab.py --n 4096 --batch 4 --arms "potrf_mode=0,potrf_lazy=1" "potrf_mode=1,potrf_lazy=2"  (fit_batched)
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
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--d", type=int, default=8)
ap.add_argument("--kernel", default="rbf")
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--arms", nargs="+", default=["potrf_half=0", "potrf_half=-1"])
a = ap.parse_args()

dev = torch.device("cuda", 0)
eng = GPEngine(dev)
p = KernelParams(a.kernel, botorch_default_lengthscale(a.d), noise=1e-4)
if a.batch > 1:
    probs = [synthetic.problem(a.n, a.d, s) for s in range(a.batch)]
    Xt = torch.stack([torch.tensor(X, device=dev) for X, _ in probs])
    yt = torch.stack([torch.tensor(y, device=dev) for _, y in probs])


    class _States(list):  # the problems' states, plus their stacked alpha for the bitwise comparison
        pass

    def fit(check, out):
        sts = _States(eng.fit_batched(Xt, yt, p, check=check, out=out))
        sts.alpha = torch.stack([s.alpha for s in sts])
        return sts
else:
    X, y = synthetic.problem(a.n, a.d, 0)
    Xt, yt = torch.tensor(X, device=dev), torch.tensor(y, device=dev)


    def fit(check, out):
        return eng.fit(Xt, yt, p, check=check, out=out)
st = fit(True, None)
torch.cuda.synchronize()
names = ["gram", "potrf", "alpha"]
eng.timing_enable(names)


def arm_opts(arm):
    out = []
    for kv in filter(None, arm.split(",")):
        k, v = kv.split("=")
        out.append((k, int(v)))
    return out


defaults = {k: eng.get_option(k) for arm in a.arms for k, _ in arm_opts(arm)}
res = {arm: [] for arm in a.arms}
parts = {arm: {k: [] for k in names} for arm in a.arms}
alpha0 = None
for rnd in range(a.rounds):
    for arm in a.arms:
        for k, v in defaults.items():
            eng.set_option(k, v)
        for k, v in arm_opts(arm):
            eng.set_option(k, v)
        st = fit(True, st)  # warm
        torch.cuda.synchronize()
        eng.timing_reset()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            st = fit(False, st)
        torch.cuda.synchronize()
        res[arm].append((time.perf_counter() - t0) / a.reps * 1e3)
        for k in names:
            ms, cnt = eng.timing_query(k)
            parts[arm][k].append(ms / max(cnt, 1))
        if rnd == 0:
            al = st.alpha.clone()
            if alpha0 is None:
                alpha0 = al
            same = bool(torch.equal(al, alpha0))
            rel = float((al - alpha0).abs().max() / alpha0.abs().max())
            print(f"arm {arm!r}: alpha bitwise equal to arm 0: {same} (max rel diff {rel:.2e}); info {int(st.info.max().item()) if a.batch == 1 else [int(x.info.item()) for x in st]}")
for arm in a.arms:
    med = statistics.median(res[arm])
    split = ", ".join(f"{k} {statistics.median(parts[arm][k]):.4f}" for k in names)
    print(f"n={a.n} {a.kernel} arm {arm!r}: update {med:.4f} ms (median of {a.rounds} rounds x {a.reps}; min "
          f"{min(res[arm]):.4f}) | {split} ms")
print("OPT AB DONE")
