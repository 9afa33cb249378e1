# A/B of two library builds (ab/libgpx_$A.so vs ab/libgpx_$B.so) on one box, alternating; then the GPU suite.
A=${1:-base}; B=${2:-nofold}
mkdir -p gpurun_out
for i in 1 2; do
  GPX_LIB=$PWD/ab/libgpx_$A.so timeout -k 10 100 python -u tools/sched_ab.py --schedules 1 > gpurun_out/ab_${A}_$i.log 2>&1 || exit 1
  GPX_LIB=$PWD/ab/libgpx_$B.so timeout -k 10 100 python -u tools/sched_ab.py --schedules 1 > gpurun_out/ab_${B}_$i.log 2>&1 || exit 1
done
grep round gpurun_out/ab_*.log
if [ -n "$3" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_full.log 2>&1; echo tests rc=$?
  tail -3 gpurun_out/tests_full.log
fi
