"""A/B of libgpx builds: run the same command once per library per round, alternating (GPX_LIB selects the library),
and report the median of every number a regex extracts.

  python tools/ab_libs.py --libs base=ab/libgpx_base.so,new=bayesianoptimizer_amd/lib/libgpx.so --rounds 5 \
      --regex 'update \\(gpx_fit_factor_f64.*?\\): ([0-9.]+) ms' -- python tools/fit_timing.py --n 4096 --kernel rbf
"""
import argparse
import os
import re
import statistics
import subprocess
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--libs", required=True, help="name=path,name=path (paths relative to the repo root)")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--regex", action="append", required=True, help="one capture group; repeatable")
ap.add_argument("--timeout", type=int, default=300)
ap.add_argument("cmd", nargs=argparse.REMAINDER)
a = ap.parse_args()
cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = dict(kv.split("=", 1) for kv in a.libs.split(","))
res = {name: [[] for _ in a.regex] for name in libs}
for r in range(a.rounds):
    for name, path in libs.items():
        env = dict(os.environ, GPX_LIB=os.path.join(root, path))
        out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=a.timeout, cwd=root)
        if out.returncode != 0:
            print(out.stdout[-2000:], out.stderr[-2000:])
            sys.exit(out.returncode)
        vals = []
        for i, rx in enumerate(a.regex):
            m = re.search(rx, out.stdout)
            if not m:
                print(f"regex {rx!r} did not match:\n{out.stdout[-2000:]}")
                sys.exit(1)
            res[name][i].append(float(m.group(1)))
            vals.append(m.group(1))
        print(f"round {r} {name}: " + " | ".join(vals), flush=True)
for name in libs:
    print(f"{name}: " + " | ".join(f"median {statistics.median(v):.4f} (min {min(v):.4f})" for v in res[name]))
print("AB DONE")
