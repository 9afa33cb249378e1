# A/B/C... of library builds ab/libgpx_<name>.so on one box, two alternating rounds (tools/sched_ab.py, multi-launch).
mkdir -p gpurun_out
for i in 1 2; do
  for v in "$@"; do
    GPX_LIB=$PWD/ab/libgpx_$v.so timeout -k 10 100 python -u tools/sched_ab.py --schedules 1 --batch 2 > gpurun_out/ab_${v}_$i.log 2>&1 || exit 1
  done
done
grep -H round gpurun_out/ab_*.log
