# K >= 384 row-major flushes: B = 8 check (g = 6 there too) and B = 4 interval re-sweep on the new order
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/ab_libs.py --libs base=ab/libgpx_base.so,rm384=bayesianoptimizer_amd/lib/libgpx.so --rounds 3 --regex "update ([0-9.]+) ms" -- python3 tools/opt_ab.py --n 4096 --batch 8 --rounds 1 --reps 5 --arms "" > gpurun_out/rm384_b8.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/opt_ab.py --n 4096 --batch 4 --rounds 4 --reps 10 --arms "" "potrf_lazy=7,potrf_mode=1,potrf_switch=50" "potrf_lazy=6,potrf_mode=1,potrf_switch=37" "potrf_lazy=6,potrf_mode=1,potrf_switch=49" > gpurun_out/rm384_b4_sweep.log 2>&1 || exit $?
