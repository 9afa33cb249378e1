# band lookahead (columns up to the next flush get column c-1 each launch) vs HEAD: fit A/B at 16384 / 8192 / 4096 and
# B = 4 batched, then the schedule-invariance tests on the new library
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
L="base=ab/libgpx_base.so,xmap=bayesianoptimizer_amd/lib/libgpx.so"
RX='update \(gpx_fit_factor_f64.*?\): ([0-9.]+) ms'
timeout -k 10 280 python3 tools/ab_libs.py --libs $L --rounds 3 --regex "$RX" -- python3 tools/fit_timing.py --n 16384 --kernel matern52 --reps 3 > gpurun_out/xmapr_16384.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/ab_libs.py --libs $L --rounds 4 --regex "$RX" -- python3 tools/fit_timing.py --n 8192 --kernel rbf --reps 5 > gpurun_out/xmapr_8192.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/ab_libs.py --libs $L --rounds 4 --regex "update ([0-9.]+) ms" -- python3 tools/opt_ab.py --n 4096 --batch 4 --rounds 3 --reps 5 --arms "" > gpurun_out/xmapr_b4.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/ab_libs.py --libs $L --rounds 5 --regex "$RX" -- python3 tools/fit_timing.py --n 4096 --kernel rbf --reps 10 > gpurun_out/xmapr_4096.log 2>&1 || exit $?
timeout -k 10 120 tools/potrf_steps_probe 16384 > gpurun_out/steps_16384_xmapr.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dataflow.py tests/test_gpu_parity.py -k "fit or potrf or chol or factor or alpha or NOT_PD or pivot or jitter or golden or configs" > gpurun_out/xmapr_tests.log 2>&1 || exit $?
