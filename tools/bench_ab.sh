#!/bin/bash
# A/B: ab/libgpx_base.so vs the working tree's libgpx, alternating short bench runs on one box; prints the trmm launch
# average (live hipEvents) and candidates/s of each run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
for i in 1 2 3 4; do
  GPX_LIB=$R/ab/libgpx_base.so timeout -k 10 200 python bench.py --no-other-configs --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/ab_base_$i.json 2>/dev/null || exit $?
  timeout -k 10 200 python bench.py --no-other-configs --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/ab_new_$i.json 2>/dev/null || exit $?
done
python3 - <<'PY'
import json, glob
for arm in ("base", "new"):
    rows = []
    for f in sorted(glob.glob(f"gpurun_out/ab_{arm}_*.json")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        rows.append((d["roofline"]["avg_launch_ms"], d["value"], d["fit_ms"]))
    print(arm, " ".join(f"trmm {a:.4f} ms / {v:.4e} c/s / fit {f:.4f}" for a, v, f in rows))
PY
echo AB DONE
