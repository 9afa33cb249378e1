# one workgroup per CU (extra dynamic LDS) for chosen Cholesky launches: n = 4096 single fit, experiment library
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export GPX_LIB=$R/ab/libgpx_x1.so
RX='update \(gpx_fit_factor_f64.*?\): ([0-9.]+) ms'
timeout -k 10 400 python3 tools/env_ab.py --rounds 4 --regex "$RX" --arms "base:" "mid:GPX_X1_LO=9,GPX_X1_HI=26" "midsplit:GPX_X1_LO=9,GPX_X1_HI=26,GPX_X1_SPLIT=1" "early:GPX_X1_LO=1,GPX_X1_HI=8" "tail:GPX_X1_LO=27,GPX_X1_HI=63" "mid2:GPX_X1_LO=9,GPX_X1_HI=20" "all:GPX_X1_LO=0,GPX_X1_HI=63" -- python3 tools/fit_timing.py --n 4096 --kernel rbf --reps 10 > gpurun_out/x1_4096.log 2>&1 || exit $?
