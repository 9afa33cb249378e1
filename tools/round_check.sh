# Full GPU check of the tree in ONE call, so every number of the round's evidence comes from the same box and tree:
#  1. rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over the sweep -> profiles/trmm_pmc_traffic.json (read by bench.py
#     for roofline.traffic) and gpurun_out/trmm_pmc_traffic.json;
#  2. an MFMA-busy pass over the Cholesky launches -> gpurun_out/potrf_mfma.json (tools/pmc_potrf.py);
#  3. the -m gpu suite, smoke, bench (N=1, P=1 and P=4);
#  4. rocprofv3 --kernel-trace --stats of the bench.
# A failing test (pytest rc 1) does not stop the measurements; a crash, abort or time limit does.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -- python3 $R/tools/sweep_only.py --m 131072 --reps 2 > $R/gpurun_out/pmc_fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -- python3 $R/tools/sweep_only.py --m 131072 --reps 2 > $R/gpurun_out/pmc_write.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_potrf -- python3 $R/tools/fit_only.py --reps 3 > $R/gpurun_out/pmc_potrf.log 2>&1 || exit $?
cd $R
python3 tools/pmc_traffic.py trmm_sumsq gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/trmm_pmc_traffic.json > gpurun_out/pmc_traffic.log 2>&1 &&
cp gpurun_out/trmm_pmc_traffic.json profiles/trmm_pmc_traffic.json &&
python3 tools/pmc_potrf.py gpurun_out/pmc_potrf 64 gpurun_out/potrf_mfma.json > gpurun_out/pmc_potrf_summary.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests ended with $rc"; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python bench.py --problems-per-gpu 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_p4.json 2> gpurun_out/bench_p4.err &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o bench --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-other-configs > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err &&
exit $rc
