# Cholesky flushes of K >= 384 in row-major tile order (B = 4 at n = 4096 on g = 6, single n = 8192 on g = 6)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
AB="python3 -u tools/ab_libs.py --libs base=ab/libgpx_base.so,rm384=bayesianoptimizer_amd/lib/libgpx.so"
timeout -k 10 300 $AB --rounds 5 --regex "arm '': update ([0-9.]+) ms" --regex "arm 'potrf_lazy=8[^']*': update ([0-9.]+) ms" -- python3 tools/opt_ab.py --n 4096 --batch 4 --rounds 1 --reps 10 --arms "" "potrf_lazy=8,potrf_mode=1,potrf_switch=49" > gpurun_out/rm384_b4.log 2>&1 || exit $?
timeout -k 10 300 $AB --rounds 4 --regex "update ([0-9.]+) ms" -- python3 tools/opt_ab.py --n 8192 --rounds 1 --reps 5 --arms "" > gpurun_out/rm384_8192.log 2>&1 || exit $?
