set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -x tests/test_gpu_parity.py tests/test_svgp.py -k "posterior or acquire or sweep or golden or svgp or configs or pool" > gpurun_out/r05_t5.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/r05_bench5.json 2> gpurun_out/r05_bench5.err
echo "bench rc=$?"
