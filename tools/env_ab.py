"""A/B of environment settings on one command: every arm runs once per round, alternating, and the median of every
number a regex extracts is reported per arm.

  python tools/env_ab.py --arms "base:" "x1:GPX_X1_LO=9,GPX_X1_HI=26" --rounds 5 \\
      --regex 'update \\(gpx_fit_factor_f64.*?\\): ([0-9.]+) ms' -- python tools/fit_timing.py --n 4096 --kernel rbf
"""
import argparse
import os
import re
import statistics
import subprocess
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--arms", nargs="+", required=True, help="name:VAR=value,VAR=value")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--regex", action="append", required=True)
ap.add_argument("--timeout", type=int, default=300)
ap.add_argument("cmd", nargs=argparse.REMAINDER)
a = ap.parse_args()
cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
arms = []
for arm in a.arms:
    name, _, kvs = arm.partition(":")
    arms.append((name, dict(kv.split("=", 1) for kv in filter(None, kvs.split(",")))))
res = {name: [[] for _ in a.regex] for name, _ in arms}
for r in range(a.rounds):
    for name, extra in arms:
        out = subprocess.run(cmd, env=dict(os.environ, **extra), capture_output=True, text=True, timeout=a.timeout,
                             cwd=root)
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
for name, _ in arms:
    print(f"{name}: " + " | ".join(f"median {statistics.median(v):.4f} (min {min(v):.4f})" for v in res[name]))
print("ENV AB DONE")
