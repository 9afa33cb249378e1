# n = 16384 per-launch trace at HEAD + the isolated flush tile bench (is the in-launch flush slower than the tile alone?)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fl
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace16 -o fit -- python3 $R/tools/fit_only.py --n 16384 --kernel matern52 --reps 2 > $O/trace16.log 2>&1 &&
cd $R && python3 tools/potrf_launches.py $O/trace16 8 > $O/launches_16384.log 2>&1 &&
timeout -k 10 120 $R/tools/flush_asm_bench 15744 512 > $O/flush_bench.log 2>&1
rc=$?
head -6 $O/launches_16384.log; tail -9 $O/flush_bench.log
exit $rc
