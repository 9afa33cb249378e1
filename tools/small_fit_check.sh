# Small-n fit latency after the dispatch trims: GPU parity suite, fit timing, kernel trace of the n = 128 fit.
set -o pipefail
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/small_fit_timing.py > gpurun_out/small_fit.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tr128b -o fit -- python3 $GRAFT_REPO_ROOT/tools/small_fit_timing.py 128 > $GRAFT_REPO_ROOT/gpurun_out/tr128b.log 2>&1
