# Round 5, call 3: hand-placed trmm in the library (+ diag skip probe), seeded trailing tiles v3 (pair loads) A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
L=base=ab/libgpx_base.so,seed2=ab/libgpx_seed2.so,new=bayesianoptimizer_amd/lib/libgpx.so
timeout -k 10 120 ./tools/trmm_asm_bench > gpurun_out/r05_trmm_asm2.log 2>&1
echo "trmm asm rc=$?"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -x tests/test_gpu_parity.py tests/test_svgp.py tests/test_gpu_small_n.py tests/test_gpu_dataflow.py > gpurun_out/r05_t3.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/r05_bench3.json 2> gpurun_out/r05_bench3.err
echo "bench rc=$?"
timeout -k 10 400 python -u tools/ab_libs.py --libs $L --rounds 5 --regex "update ([0-9.]+) ms" -- python tools/opt_ab.py --n 4096 --rounds 1 --reps 20 --arms "" > gpurun_out/r05_ab3_4096.log 2>&1 &&
timeout -k 10 400 python -u tools/ab_libs.py --libs $L --rounds 5 --regex "update ([0-9.]+) ms" -- python tools/opt_ab.py --n 4096 --batch 4 --rounds 1 --reps 10 --arms "" > gpurun_out/r05_ab3_4096_b4.log 2>&1
