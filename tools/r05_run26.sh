# TRTRI: 128-tile levels from >= 256 tiles per level (h = 16 at n = 16384, h = 32 at 8192) vs HEAD (>= 512)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
L="base=ab/libgpx_base.so,t256=ab/libgpx_t256.so"
RI='fit \+ L\^-T \(gpx_fit_f64\): ([0-9.]+) ms'
timeout -k 10 400 python3 tools/ab_libs.py --libs $L --rounds 3 --regex "$RI" -- python3 tools/fit_timing.py --n 16384 --kernel matern52 --reps 3 > gpurun_out/t256_16384.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/ab_libs.py --libs $L --rounds 4 --regex "$RI" -- python3 tools/fit_timing.py --n 8192 --kernel rbf --reps 5 > gpurun_out/t256_8192.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/ab_libs.py --libs $L --rounds 4 --regex "$RI" -- python3 tools/fit_timing.py --n 4096 --kernel rbf --reps 10 > gpurun_out/t256_4096.log 2>&1 || exit $?
