# MLL gradient on the hand-placed tile vs HEAD (MfmaTile): timing A/B and the MLL tests (bit-identical expected)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
L="base=ab/libgpx_base.so,asm=bayesianoptimizer_amd/lib/libgpx.so"
timeout -k 10 400 python3 tools/ab_libs.py --libs $L --rounds 3 --regex 'n=4096 rbf: mll value\+grad ([0-9.]+) ms' --regex 'n=4096 scale_linear_matern52: mll value\+grad ([0-9.]+) ms' --regex 'n=16384 rbf: mll value\+grad ([0-9.]+) ms' --regex 'nll (-?[0-9.]+)\)' -- python3 tools/mll_kernel_timing.py 1024 4096 16384 > gpurun_out/mll_asm_ab.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mll.py -m gpu > gpurun_out/mll_asm_tests.log 2>&1 || exit $?
