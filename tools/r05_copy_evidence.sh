#!/bin/bash
# Copy the outputs of tools/r05_evidence.sh (gpurun_out/ev) into profiles/ under their round-5 names.
set -e
cd "$(dirname "$0")/.."
[ -s gpurun_out/ev/bench.json ] && [ -s gpurun_out/ev/bench_p4.json ] || { echo "no complete evidence set in gpurun_out/ev"; exit 1; }
E=gpurun_out/ev
tail -n 1 $E/bench.json > profiles/r05_bench_line.json
tail -n 1 $E/bench_p4.json > profiles/r05_bench_line_p4.json
cp "$(ls $E/prof/*kernel_stats.csv | head -1)" profiles/r05_bench_kernel_stats.csv
cp $E/trmm_pmc_traffic.json profiles/r05_trmm_pmc_traffic.json
cp $E/trmm_pmc_traffic.json profiles/trmm_pmc_traffic.json
cp $E/trmm_pmc_sq.json profiles/r05_trmm_pmc_sq.json
cp $E/potrf_mfma.json profiles/r05_pmc_potrf_mfma.json
cp $E/potrf_launches_4096.log profiles/r05_potrf_launches_4096.log
grep -v "amdgpu.ids" $E/gpu_tests.log > profiles/r05_gpu_tests.log
grep -v "amdgpu.ids" $E/smoke.log > profiles/r05_smoke.log
echo "copied"
