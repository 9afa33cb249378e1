# batched lookahead switch after the flush at nblk - 16 for B >= 4 (B = 4 / 8 at n = 4096), B = 2 unchanged
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
AB="python3 -u tools/ab_libs.py --libs base=ab/libgpx_base.so,sw49=bayesianoptimizer_amd/lib/libgpx.so"
timeout -k 10 300 $AB --rounds 5 --regex "update ([0-9.]+) ms" -- python3 tools/opt_ab.py --n 4096 --batch 4 --rounds 1 --reps 10 --arms "" > gpurun_out/sw49_b4.log 2>&1 || exit $?
timeout -k 10 300 $AB --rounds 4 --regex "update ([0-9.]+) ms" -- python3 tools/opt_ab.py --n 4096 --batch 8 --rounds 1 --reps 5 --arms "" > gpurun_out/sw49_b8.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dataflow.py tests/test_gpu_parity.py -m gpu -k "batch or schedule or configs3" > gpurun_out/sw49_tests.log 2>&1 || exit $?
