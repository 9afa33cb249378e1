# sweep product: row tiles paired (nI/2 + l, nI/2 - 1 - l) per workgroup: bench A/B + the parity suite
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python3 -u tools/ab_libs.py --libs base=ab/libgpx_base.so,pair=bayesianoptimizer_amd/lib/libgpx.so --rounds 3 --timeout 240 --regex '"avg_launch_ms": ([0-9.]+), "launches": [0-9]+, "flops_per_launch"' --regex '"value": ([0-9.e+]+)' --regex '"best": {"value": [-0-9.e]+, "index": ([0-9]+)' -- python3 bench.py --steps 5 --warmup 2 --no-other-configs --no-cpu-baseline > gpurun_out/pair_ab.log 2>&1 || exit $?
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_svgp.py -m gpu > gpurun_out/pair_tests.log 2>&1 || exit $?
