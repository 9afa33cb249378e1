set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_svgp.py -m gpu -k fps > gpurun_out/fps_edge_tests.log 2>&1 || exit $?
