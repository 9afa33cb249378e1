set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -x tests/test_gpu_parity.py -k "trtri or large_fit or configs2 or alpha or append" tests/test_append.py > gpurun_out/r05_t6.log 2>&1
echo "tests rc=$?"
timeout -k 10 500 python -u tools/ab_libs.py --libs base=ab/libgpx_base.so,new=bayesianoptimizer_amd/lib/libgpx.so --rounds 3 --regex "\(gpx_fit_f64\): ([0-9.]+) ms" --regex "gpx_fit_f64\).*trtri ([0-9.]+) ms" -- python tools/fit_timing.py --n 16384 --reps 2 > gpurun_out/r05_ab6_16384.log 2>&1
echo "ab rc=$?"
timeout -k 10 300 python -u tools/ab_libs.py --libs base=ab/libgpx_base.so,new=bayesianoptimizer_amd/lib/libgpx.so --rounds 3 --regex "gpx_fit_f64\).*trtri ([0-9.]+) ms" -- python tools/fit_timing.py --n 8192 --kernel rbf --reps 3 > gpurun_out/r05_ab6_8192.log 2>&1
