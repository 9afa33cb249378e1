# A/B of library builds at a large n (tools/sched_ab.py, multi-launch), alternating; N = $1, then the builds.
N=$1; shift
mkdir -p gpurun_out
for i in 1 2; do
  for v in "$@"; do
    GPX_LIB=$PWD/ab/libgpx_$v.so timeout -k 10 150 python -u tools/sched_ab.py --n $N --schedules 1 --batch 1 --reps 4 > gpurun_out/abL_${N}_${v}_$i.log 2>&1 || exit 1
  done
done
grep -H "round 1" gpurun_out/abL_*.log
