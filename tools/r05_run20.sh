# 16-block diagonal skip in the sweep product (tail8): probe (bit-exact vs MfmaTile), bench A/B vs HEAD, sweep parity
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 120 tools/trmm_asm_bench 4096 32768 > gpurun_out/tail8b_probe.log 2>&1 || exit $?
timeout -k 10 500 python3 tools/ab_libs.py --libs base=ab/libgpx_base.so,tail8=bayesianoptimizer_amd/lib/libgpx.so --rounds 3 --timeout 240 --regex '"value": ([0-9.e+]+)' --regex '"roofline": {[^}]*"frac": ([0-9.]+)' --regex '"best": {"value": [^,]*, "index": ([0-9]+)' -- python3 bench.py --steps 5 --warmup 2 --no-other-configs --no-cpu-baseline > gpurun_out/tail8b_bench.log 2>&1 || exit $?
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_realdata.py tests/test_gpu_small_n.py > gpurun_out/tail8b_tests.log 2>&1 || exit $?
