# single n = 4096 fit: early lookahead interval 3 / 5 with the switch after its flushes, against the default (g = 4, switch 9)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/opt_ab.py --n 4096 --rounds 6 --reps 20 --arms "" "potrf_switch=10,potrf_lazy=3" "potrf_switch=7,potrf_lazy=3" "potrf_switch=13,potrf_lazy=3" "potrf_switch=11,potrf_lazy=5" "potrf_switch=6,potrf_lazy=5" > gpurun_out/early_g_4096.log 2>&1 || exit $?
