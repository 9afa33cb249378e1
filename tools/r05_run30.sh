# register-resident FPS: SVGP parity tests (FPS bit-exact vs the oracle) and the pool-scan timing
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_svgp.py tests/test_dropin_gpu.py > gpurun_out/fps_tests.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/svgp_scan_only.py > gpurun_out/fps_scan.log 2>&1 || exit $?
