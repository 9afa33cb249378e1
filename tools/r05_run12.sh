# L capture off the pivot chain: A/B vs HEAD library (fit_timing), then the dataflow/parity tests that pin the factor
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ab_libs.py --libs base=ab/libgpx_base.so,new=bayesianoptimizer_amd/lib/libgpx.so --rounds 5 --regex 'update \(gpx_fit_factor_f64.*?\): ([0-9.]+) ms' -- python3 tools/fit_timing.py --n 4096 --kernel rbf > gpurun_out/lcap_ab.log 2>&1 || exit $?
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dataflow.py tests/test_gpu_parity.py -k "fit or potrf or chol or factor or alpha or NOT_PD or pivot or jitter or golden or configs" > gpurun_out/lcap_tests.log 2>&1 || exit $?
