# flush launches (K >= 256) in row-major tile order (xmap 0) vs the XCD-chunked 8x8 super-block order (xmap 1)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export GPX_LIB=$R/ab/libgpx_xx.so
RX='update \(gpx_fit_factor_f64.*?\): ([0-9.]+) ms'
timeout -k 10 400 python3 tools/env_ab.py --rounds 3 --regex "$RX" --arms "x1:GPX_X_XMAP=1" "x0:GPX_X_XMAP=0" -- python3 tools/fit_timing.py --n 16384 --kernel matern52 --reps 3 > gpurun_out/xx_16384.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/env_ab.py --rounds 4 --regex "$RX" --arms "x1:GPX_X_XMAP=1" "x0:GPX_X_XMAP=0" -- python3 tools/fit_timing.py --n 8192 --kernel rbf --reps 5 > gpurun_out/xx_8192.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/env_ab.py --rounds 4 --regex "update ([0-9.]+) ms" --arms "x1:GPX_X_XMAP=1" "x0:GPX_X_XMAP=0" -- python3 tools/opt_ab.py --n 4096 --batch 4 --rounds 3 --reps 5 --arms "" > gpurun_out/xx_b4.log 2>&1 || exit $?
