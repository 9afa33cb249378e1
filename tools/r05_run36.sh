# Gram centring by the row block's first row: bench A/B (gram kernel live time, value) and the full GPU suite
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python3 tools/ab_libs.py --libs base=ab/libgpx_base.so,kfirst=bayesianoptimizer_amd/lib/libgpx.so --rounds 3 --timeout 240 --regex '"kernel_build_roofline": {[^}]*"avg_launch_ms": ([0-9.]+)' --regex '"fit_ms": ([0-9.]+)' --regex '"value": ([0-9.e+]+)' -- python3 bench.py --steps 5 --warmup 2 --no-other-configs --no-cpu-baseline > gpurun_out/kfirst_ab.log 2>&1 || exit $?
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/kfirst_tests.log 2>&1 || exit $?
