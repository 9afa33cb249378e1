#!/bin/bash
# A/B of libgpx builds on the bench step: alternating short bench runs on one box, one per library per round; prints
# the trmm launch average (live hipEvents), candidates/s and fit time of each run.  Arguments: name=path (relative to
# the repo root; "name=" = the working tree's library); default: base=ab/libgpx_base.so new=
#   bash tools/bench_ab.sh base=ab/libgpx_base.so head=ab/libgpx_head.so new=
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
[ $# -eq 0 ] && set -- base=ab/libgpx_base.so new=
rm -f gpurun_out/ab_*_*.json
for i in 1 2 3 4; do
  for arm in "$@"; do
    name=${arm%%=*}; lib=${arm#*=}
    if [ -n "$lib" ]; then export GPX_LIB=$R/$lib; else unset GPX_LIB; fi
    timeout -k 10 200 python bench.py --no-other-configs --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/ab_${name}_$i.json 2>/dev/null || exit $?
  done
done
unset GPX_LIB
python3 - "$@" <<'PY'
import json, glob, sys, statistics
for arm in sys.argv[1:]:
    name = arm.split("=", 1)[0]
    rows = []
    for f in sorted(glob.glob(f"gpurun_out/ab_{name}_*.json")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        rows.append((d["roofline"]["avg_launch_ms"], d["value"], d["fit_ms"]))
    print(f"{name}: trmm median {statistics.median(r[0] for r in rows):.4f} ms |",
          " ".join(f"{a:.4f}/{v:.4e}/{f:.4f}" for a, v, f in rows))
PY
echo AB DONE
