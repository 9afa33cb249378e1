# kernel stats of the n = 16384 fit + inverse (trtri T vs W12 products per level)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/trace19
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace19 -o fit -- python3 $R/tools/fit_timing.py --n 16384 --kernel matern52 --reps 2 > $R/gpurun_out/trace19.log 2>&1 || exit $?
