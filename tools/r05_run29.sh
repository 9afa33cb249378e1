# SVGP pool-scan kernel trace (scoring vs top-k vs FPS)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/trace29
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace29 -o scan -- python3 $R/tools/svgp_scan_only.py > $R/gpurun_out/trace29.log 2>&1 || exit $?
