# Round 5, call 1: the schedule-invariant trailing update, real-data parity, timeout fallback; A/B against HEAD~ (base).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -x tests/test_gpu_realdata.py tests/test_gpu_dataflow.py "tests/test_gpu_parity.py::test_configs3_selection_independent_of_problems_per_gpu" "tests/test_gpu_parity.py::test_fit_batched_potrs_multiblock_owners" "tests/test_gpu_parity.py::test_configs3_per_gpu_share_batched_n4096" tests/test_dropin_gpu.py -s > gpurun_out/r05_t1.log 2>&1
rc=$?
echo "targeted tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/ab_libs.py --libs base=ab/libgpx_base.so,new=bayesianoptimizer_amd/lib/libgpx.so --rounds 5 --regex "update ([0-9.]+) ms" -- python tools/opt_ab.py --n 4096 --rounds 1 --reps 20 --arms "" > gpurun_out/r05_ab_4096.log 2>&1 &&
timeout -k 10 400 python -u tools/ab_libs.py --libs base=ab/libgpx_base.so,new=bayesianoptimizer_amd/lib/libgpx.so --rounds 5 --regex "update ([0-9.]+) ms" -- python tools/opt_ab.py --n 4096 --batch 4 --rounds 1 --reps 10 --arms "" > gpurun_out/r05_ab_4096_b4.log 2>&1 &&
timeout -k 10 400 python -u tools/ab_libs.py --libs base=ab/libgpx_base.so,new=bayesianoptimizer_amd/lib/libgpx.so --rounds 3 --regex "update ([0-9.]+) ms" -- python tools/opt_ab.py --n 16384 --kernel matern52 --rounds 1 --reps 3 --arms "" > gpurun_out/r05_ab_16384.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05_gpu_tests.log 2>&1
rc=$?
echo "full gpu suite rc=$rc"
exit $rc
