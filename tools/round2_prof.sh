# Round-2 profile pass: kernel trace + stats of a short bench run, and the Cholesky MFMA-busy counter pass.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o bench --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-other-configs > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err &&
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/pmc_potrf -- python3 $R/tools/fit_only.py --n 4096 --reps 3 > $R/gpurun_out/pmc_potrf.log 2>&1 &&
cd $R && python3 tools/pmc_potrf.py gpurun_out/pmc_potrf 64 gpurun_out/r02_pmc_potrf_mfma.json > gpurun_out/pmc_potrf_summary.log 2>&1
