# Round 5, call 2: seeded trailing tiles v2 (row-major first k-tile) A/B against round 4 (base) and v1 (seed1);
# hand-placed trmm probe; invariance + batched tests on the new library.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
L=base=ab/libgpx_base.so,seed1=ab/libgpx_seed1.so,new=bayesianoptimizer_amd/lib/libgpx.so
timeout -k 10 120 ./tools/trmm_asm_bench > gpurun_out/r05_trmm_asm.log 2>&1
echo "trmm asm rc=$?"
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -x tests/test_gpu_dataflow.py -k "identical or not_pd" "tests/test_gpu_parity.py::test_configs3_selection_independent_of_problems_per_gpu" "tests/test_gpu_parity.py::test_fit_batched_matches_single_fits_and_oracle" "tests/test_gpu_parity.py::test_potrs_alpha_matches_inverse_path_and_oracle" > gpurun_out/r05_t2.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_libs.py --libs $L --rounds 5 --regex "update ([0-9.]+) ms" -- python tools/opt_ab.py --n 4096 --rounds 1 --reps 20 --arms "" > gpurun_out/r05_ab2_4096.log 2>&1 &&
timeout -k 10 400 python -u tools/ab_libs.py --libs $L --rounds 5 --regex "update ([0-9.]+) ms" -- python tools/opt_ab.py --n 4096 --batch 4 --rounds 1 --reps 10 --arms "" > gpurun_out/r05_ab2_4096_b4.log 2>&1 &&
timeout -k 10 500 python -u tools/ab_libs.py --libs $L --rounds 3 --regex "update ([0-9.]+) ms" -- python tools/opt_ab.py --n 16384 --kernel matern52 --rounds 1 --reps 3 --arms "" > gpurun_out/r05_ab2_16384.log 2>&1
