#!/bin/bash
# Sweep-chunk sweep: GPX_SWEEP_CHUNK_MB (K* byte budget) x GPX_SWEEP_CHUNK_MAX (candidate cap); n=4096, 2^20 cands.
set -e
for cfg in "256 16384" "512 16384" "1024 32768" "2048 65536" "512 16384" "1024 32768"; do
  set -- $cfg
  GPX_SWEEP_CHUNK_MB=$1 GPX_SWEEP_CHUNK_MAX=$2 timeout -k 10 200 python bench.py --no-other-configs --no-cpu-baseline > gpurun_out/chunk_$1.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/chunk_$1.json')); print('chunk_mb=$1 max=$2', round(d['value']), 'trmm_ms', round(d['roofline']['avg_launch_ms'],4), 'launches', d['roofline']['launches'], 'TF', round(d['roofline']['achieved'],2), 'kstar GB/s', round(d['kernel_build_roofline']['achieved']))"
done
