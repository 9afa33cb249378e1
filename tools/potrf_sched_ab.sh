#!/bin/bash
# Cholesky flush-schedule A/B at n = $1 (default 4096): for each "MODE:LAZY:EARLY_G:EARLY_END" config (empty = library
# default), the per-launch timeline probe twice, alternating; then tools/fit_timing.py per config.
set -o pipefail
N=${1:-4096}
shift
CONFIGS=${@:-":::"}
mkdir -p gpurun_out/sched
run_env() {
  IFS=: read -r M L G E <<< "$1"
  env ${M:+GPX_POTRF_MODE=$M} ${L:+GPX_POTRF_LAZY=$L} ${G:+GPX_POTRF_EARLY_G=$G} ${E:+GPX_POTRF_EARLY_END=$E} "${@:2}"
}
for i in 1 2; do
  for cfg in $CONFIGS; do
    tag=$(echo "$cfg" | tr ':' '_')
    run_env "$cfg" timeout -k 10 60 tools/potrf_steps_probe $N > gpurun_out/sched/n${N}_${tag}_$i.log 2>&1 || exit 1
  done
done
for cfg in $CONFIGS; do
  tag=$(echo "$cfg" | tr ':' '_')
  run_env "$cfg" timeout -k 10 120 python tools/fit_timing.py --n $N --kernel rbf --reps 30 > gpurun_out/sched/fit_n${N}_${tag}.log 2>&1 || exit 1
done
echo SCHED AB DONE
