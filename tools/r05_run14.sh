# per-launch trace of the n = 16384 factorisation with the band-lookahead library
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/trace14
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace14 -o fit -- python3 $R/tools/fit_only.py --n 16384 --kernel matern52 --reps 2 > $R/gpurun_out/trace14.log 2>&1 || exit $?
cd $R
python3 tools/potrf_launches.py gpurun_out/trace14 8 > gpurun_out/band_launches_16384.log 2>&1
