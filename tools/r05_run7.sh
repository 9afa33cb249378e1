set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
L=base=ab/libgpx_base.so,seed2=ab/libgpx_seed2.so,new=bayesianoptimizer_amd/lib/libgpx.so
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -x tests/test_gpu_dataflow.py tests/test_gpu_parity.py -k "potrf or not_pd or identical or batched or configs3 or potrs or large_fit or lookahead" > gpurun_out/r05_t7.log 2>&1
echo "tests rc=$?"
timeout -k 10 400 python -u tools/ab_libs.py --libs $L --rounds 5 --regex "update ([0-9.]+) ms" -- python tools/opt_ab.py --n 4096 --rounds 1 --reps 20 --arms "" > gpurun_out/r05_ab7_4096.log 2>&1 &&
timeout -k 10 400 python -u tools/ab_libs.py --libs $L --rounds 5 --regex "update ([0-9.]+) ms" -- python tools/opt_ab.py --n 4096 --batch 4 --rounds 1 --reps 10 --arms "" > gpurun_out/r05_ab7_4096_b4.log 2>&1 &&
timeout -k 10 500 python -u tools/ab_libs.py --libs $L --rounds 3 --regex "update ([0-9.]+) ms" -- python tools/opt_ab.py --n 16384 --kernel matern52 --rounds 1 --reps 3 --arms "" > gpurun_out/r05_ab7_16384.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py --libs $L --rounds 3 --regex "update ([0-9.]+) ms" -- python tools/opt_ab.py --n 8192 --rounds 1 --reps 5 --arms "" > gpurun_out/r05_ab7_8192.log 2>&1
