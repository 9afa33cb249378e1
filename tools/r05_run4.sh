# Round 5, call 4: SQ counters of the hand-placed sweep product (library, sweep_only) and of the probe variants.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $C1 --output-format csv -d $R/gpurun_out/pmc4_lib -- python3 $R/tools/sweep_only.py --m 131072 --reps 2 > $R/gpurun_out/pmc4_lib.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc $C1 --output-format csv -d $R/gpurun_out/pmc4_probe -- $R/tools/trmm_asm_bench > $R/gpurun_out/pmc4_probe.log 2>&1 || exit $?
cd $R
for k in trmm_sumsq_kernel; do python3 tools/pmc_summary.py $k gpurun_out/pmc4_lib --out gpurun_out/pmc4_lib_$k.json; done > gpurun_out/pmc4_summary.log
for v in 0 1 2; do python3 tools/pmc_summary.py "trmm_vILi${v}" gpurun_out/pmc4_probe --out gpurun_out/pmc4_probe_$v.json; done >> gpurun_out/pmc4_summary.log
echo PMC4 DONE
