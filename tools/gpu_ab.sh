# One A/B measurement or probe on the GPU box, output to gpurun_out/LOG.log (replaces round 5's one-off run scripts):
#   gpurun --timeout 600 -- 'bash tools/gpu_ab.sh early_g_4096 400 python3 -u tools/opt_ab.py --n 4096 --arms "" "potrf_lazy=3"'
# The command runs under its own time limit; a crash, abort or time limit ends the call with that status.
set -o pipefail
log=$1
secs=$2
shift 2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out || exit 1
timeout -k 10 "$secs" "$@" > "gpurun_out/$log.log" 2>&1
rc=$?
tail -5 "gpurun_out/$log.log"
exit $rc
