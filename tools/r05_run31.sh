# MLL value + gradient timing (n = 1024 / 4096 / 16384) and its kernel split
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/trace31
cd $R && timeout -k 10 200 python3 tools/mll_kernel_timing.py 1024 4096 16384 > gpurun_out/mll_timing.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace31 -o mll -- python3 $R/tools/mll_kernel_timing.py 4096 > $R/gpurun_out/trace31.log 2>&1 || exit $?
