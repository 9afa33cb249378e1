# Full GPU check of the tree: parity suite, smoke, bench (N=1, P=1 and P=4), rocprofv3 kernel stats of the bench,
# FETCH_SIZE / WRITE_SIZE passes over the sweep -> per-launch HBM traffic of trmm_sumsq (tools/pmc_traffic.py).
# A failing test (pytest rc 1) does not stop the measurements; a crash, abort or time limit does.
set -o pipefail
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests ended with $rc"; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python bench.py --problems-per-gpu 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_p4.json 2> gpurun_out/bench_p4.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-other-configs > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_bench.err &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_fetch -- python3 $GRAFT_REPO_ROOT/tools/sweep_only.py --m 131072 --reps 2 > $GRAFT_REPO_ROOT/gpurun_out/pmc_fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_write -- python3 $GRAFT_REPO_ROOT/tools/sweep_only.py --m 131072 --reps 2 > $GRAFT_REPO_ROOT/gpurun_out/pmc_write.log 2>&1 &&
cd $GRAFT_REPO_ROOT && python3 tools/pmc_traffic.py trmm_sumsq gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/trmm_pmc_traffic.json > gpurun_out/pmc_traffic.log 2>&1 &&
exit $rc
