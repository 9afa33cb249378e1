# The round's evidence set, ONE call, one box, one tree (profiles/README.md indexes the outputs; tools/copy_evidence.sh
# ROUND copies them into profiles/ under the round's names):
#  1. rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over the sweep -> trmm HBM traffic (bench.py roofline.traffic);
#  2. SQ pass over the sweep product (MFMA busy per SIMD, wave-cycle split) and the Cholesky's MFMA-busy per launch;
#  3. per-launch kernel trace of the n = 4096 update, and the per-phase timeline of its launches (tools/potrf_steps_probe,
#     built in-tree beforehand: launch gap, pre-update, the four 16-pivot blocks, factor tail, store);
#  4. the -m gpu suite, smoke, bench (N=1), bench --problems-per-gpu 4;
#  5. rocprofv3 --kernel-trace --stats of the bench.
# A failing test (pytest rc 1) does not stop the measurements; a crash, abort or time limit does.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ev
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -- python3 $R/tools/sweep_only.py --m 131072 --reps 2 > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -- python3 $R/tools/sweep_only.py --m 131072 --reps 2 > $O/pmc_write.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq -- python3 $R/tools/sweep_only.py --m 131072 --reps 2 > $O/pmc_sq.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_potrf -- python3 $R/tools/fit_only.py --reps 3 > $O/pmc_potrf.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o fit -- python3 $R/tools/fit_only.py --n 4096 --reps 3 > $O/trace.log 2>&1 &&
timeout -k 10 120 $R/tools/potrf_steps_probe 4096 0 1 > $O/potrf_steps_4096.log 2>&1 || exit $?
cd $R
python3 tools/pmc_traffic.py trmm_sumsq $O/pmc_fetch $O/pmc_write $O/trmm_pmc_traffic.json > $O/pmc_traffic.log 2>&1 &&
cp $O/trmm_pmc_traffic.json profiles/trmm_pmc_traffic.json &&
python3 tools/pmc_summary.py trmm_sumsq $O/pmc_sq --out $O/trmm_pmc_sq.json > /dev/null &&
python3 tools/pmc_potrf.py $O/pmc_potrf 64 $O/potrf_mfma.json > $O/pmc_potrf_summary.log 2>&1 &&
python3 tools/potrf_launches.py $O/trace 8 > $O/potrf_launches_4096.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests ended with $rc"; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py --problems-per-gpu 4 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_p4.json 2> $O/bench_p4.err &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-other-configs > $O/prof_bench.json 2> $O/prof_bench.err || exit $?
echo "EVIDENCE DONE rc=$rc"
exit $rc
