# diagonal-block inverses folded into the step launches: A/B vs HEAD (n = 4096 single / B = 4 / n = 16384), full GPU suite
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
L="base=ab/libgpx_base.so,dinv=bayesianoptimizer_amd/lib/libgpx.so"
RX='update \(gpx_fit_factor_f64.*?\): ([0-9.]+) ms'
RI='fit \+ L\^-T \(gpx_fit_f64\): ([0-9.]+) ms'
timeout -k 10 250 python3 tools/ab_libs.py --libs $L --rounds 5 --regex "$RX" --regex "$RI" -- python3 tools/fit_timing.py --n 4096 --kernel rbf --reps 10 > gpurun_out/dinv_4096.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/ab_libs.py --libs $L --rounds 4 --regex "update ([0-9.]+) ms" -- python3 tools/opt_ab.py --n 4096 --batch 4 --rounds 3 --reps 5 --arms "" > gpurun_out/dinv_b4.log 2>&1 || exit $?
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/dinv_tests.log 2>&1 || exit $?
