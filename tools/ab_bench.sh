#!/bin/bash
# A/B: baseline libgpx (ab/libgpx_base.so) vs the working tree's, alternating bench runs on one box.
set -e
for i in 1 2; do
  GPX_LIB=$PWD/ab/libgpx_base.so timeout -k 10 200 python bench.py --no-other-configs --no-cpu-baseline > gpurun_out/ab_base_$i.json 2>/dev/null
  timeout -k 10 200 python bench.py --no-other-configs --no-cpu-baseline > gpurun_out/ab_new_$i.json 2>/dev/null
done
echo AB DONE
