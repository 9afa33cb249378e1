set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06a/gpu_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-other-configs > gpurun_out/r06a/bench.json 2> gpurun_out/r06a/bench.err
rc=$?
tail -3 gpurun_out/r06a/gpu_tests.log
exit $rc
