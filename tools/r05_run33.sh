# Gram row split (GPX_OPT_GRAM_SPLIT) re-measured after the first-row centring
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 200 python3 tools/opt_ab.py --n 4096 --rounds 5 --reps 10 --arms "" "gram_split=2" "gram_split=4" > gpurun_out/gram_split_4096.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/opt_ab.py --n 16384 --kernel matern52 --rounds 2 --reps 2 --arms "" "gram_split=2" > gpurun_out/gram_split_16384.log 2>&1 || exit $?
