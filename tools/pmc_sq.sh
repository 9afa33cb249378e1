#!/bin/bash
# SQ stall breakdown for the sweep kernels (one --pmc pass each; guide MI355X_MICROARCH.md "rocprofv3 PMC slots").
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $R/gpurun_out/pmc_list.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/pmc_sq -- python3 $R/tools/sweep_only.py --m 131072 --reps 2 > $R/gpurun_out/pmc_sq.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_LDS_UNALIGNED_STALL --output-format csv -d $R/gpurun_out/pmc_sq2 -- python3 $R/tools/sweep_only.py --m 131072 --reps 2 > $R/gpurun_out/pmc_sq2.log 2>&1
echo PMC DONE
