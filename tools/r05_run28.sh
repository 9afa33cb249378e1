# row-major flush order only for K >= 512 (new) vs K >= 256 (HEAD)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
L="base=ab/libgpx_base.so,k512=bayesianoptimizer_amd/lib/libgpx.so"
RX='update \(gpx_fit_factor_f64.*?\): ([0-9.]+) ms'
timeout -k 10 250 python3 tools/ab_libs.py --libs $L --rounds 5 --regex "$RX" -- python3 tools/fit_timing.py --n 4096 --kernel rbf --reps 10 > gpurun_out/k512_4096.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/ab_libs.py --libs $L --rounds 4 --regex "$RX" -- python3 tools/fit_timing.py --n 8192 --kernel rbf --reps 5 > gpurun_out/k512_8192.log 2>&1 || exit $?
