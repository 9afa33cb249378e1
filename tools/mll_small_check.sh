# Hyperparameter-fit timing at small n (the reference's own BO sizes) and a kernel trace of the n = 128 evaluations,
# after the MLL GPU parity tests.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_mll.py tests/test_dropin_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/mll_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/mll_timing.py 64,128,256,1024 > gpurun_out/mll_small.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/trmll -o mll -- python3 $GRAFT_REPO_ROOT/tools/mll_timing.py 128 > $GRAFT_REPO_ROOT/gpurun_out/trmll.log 2>&1
