# trtri: groups interleaved with the heavy tiles first (128-tile levels) vs HEAD; inverse A/B at 16384 / 8192, tests
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
L="base=ab/libgpx_base.so,inter=bayesianoptimizer_amd/lib/libgpx.so"
RI='fit \+ L\^-T \(gpx_fit_f64\): ([0-9.]+) ms.*?trtri ([0-9.]+) ms'
timeout -k 10 400 python3 tools/ab_libs.py --libs $L --rounds 3 --regex "$RI" -- python3 tools/fit_timing.py --n 16384 --kernel matern52 --reps 3 > gpurun_out/trtri_inter_16384.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/ab_libs.py --libs $L --rounds 4 --regex "$RI" -- python3 tools/fit_timing.py --n 8192 --kernel rbf --reps 5 > gpurun_out/trtri_inter_8192.log 2>&1 || exit $?
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_append.py tests/test_mll.py -m gpu > gpurun_out/trtri_inter_tests.log 2>&1 || exit $?
