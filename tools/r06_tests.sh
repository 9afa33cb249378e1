# -m gpu tests on the box: the named test files first (verbose), then the whole suite
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06t
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu "$@" > gpurun_out/r06t/first.log 2>&1
rc=$?
tail -15 gpurun_out/r06t/first.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r06t/all.log 2>&1
rc=$?
tail -15 gpurun_out/r06t/all.log
exit $rc
