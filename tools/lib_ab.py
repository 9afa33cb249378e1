"""A/B of two libgpx builds on the posterior update: run as two processes per round (GPX_LIB selects the library),
alternating, each printing its update time; this driver reports the medians.

  python tools/lib_ab.py --base ab/libgpx_base.so --n 4096 --kernel rbf --rounds 5
"""
import argparse
import os
import re
import statistics
import subprocess
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--base", default="ab/libgpx_base.so")
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--kernel", default="rbf")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
arms = {"base": os.path.join(root, a.base), "new": os.path.join(root, "bayesianoptimizer_amd", "lib", "libgpx.so")}
res = {k: [] for k in arms}
split = {k: [] for k in arms}
for r in range(a.rounds):
    for name, lib in arms.items():
        env = dict(os.environ, GPX_LIB=lib)
        out = subprocess.run([sys.executable, os.path.join(root, "tools", "opt_ab.py"), "--n", str(a.n), "--kernel",
                              a.kernel, "--rounds", "1", "--reps", str(a.reps), "--arms", "spin_limit=4194304"],
                             env=env, capture_output=True, text=True, timeout=600)
        m = re.search(r"update ([0-9.]+) ms .*\| (.*) ms", out.stdout)
        if not m:
            print(out.stdout, out.stderr)
            sys.exit(1)
        res[name].append(float(m.group(1)))
        split[name].append(m.group(2))
        print(f"round {r} {name}: {m.group(1)} ms | {m.group(2)}", flush=True)
for name in arms:
    print(f"n={a.n} {a.kernel} {name}: update median {statistics.median(res[name]):.4f} ms (min {min(res[name]):.4f})")
print("LIB AB DONE")
