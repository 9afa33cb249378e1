#!/bin/bash
# Copy the outputs of tools/evidence.sh (gpurun_out/ev) into profiles/ under the round's names: tools/copy_evidence.sh r06
set -e
R=${1:?round tag, e.g. r06}
cd "$(dirname "$0")/.."
[ -s gpurun_out/ev/bench.json ] && [ -s gpurun_out/ev/bench_p4.json ] || { echo "no complete evidence set in gpurun_out/ev"; exit 1; }
E=gpurun_out/ev
tail -n 1 $E/bench.json > profiles/${R}_bench_line.json
tail -n 1 $E/bench_p4.json > profiles/${R}_bench_line_p4.json
cp "$(ls $E/prof/*kernel_stats.csv | head -1)" profiles/${R}_bench_kernel_stats.csv
cp $E/trmm_pmc_traffic.json profiles/${R}_trmm_pmc_traffic.json
cp $E/trmm_pmc_traffic.json profiles/trmm_pmc_traffic.json
cp $E/trmm_pmc_sq.json profiles/${R}_trmm_pmc_sq.json
cp $E/potrf_mfma.json profiles/${R}_pmc_potrf_mfma.json
cp $E/potrf_launches_4096.log profiles/${R}_potrf_launches_4096.log
cp $E/potrf_steps_4096.log profiles/${R}_potrf_steps_4096.log
grep -v "amdgpu.ids" $E/gpu_tests.log > profiles/${R}_gpu_tests.log
grep -v "amdgpu.ids" $E/smoke.log > profiles/${R}_smoke.log
echo "copied"
