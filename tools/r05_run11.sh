# staggered flush schedule (potrf_mode=2) A/B against the default schedules; alpha must stay bit-identical
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 150 python3 tools/opt_ab.py --n 4096 --rounds 5 --reps 10 --arms "" "potrf_mode=2,potrf_lazy=2" "potrf_mode=2,potrf_lazy=3" "potrf_mode=2,potrf_lazy=4" "potrf_mode=2,potrf_lazy=1" > gpurun_out/stag_4096.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/opt_ab.py --n 16384 --kernel matern52 --rounds 2 --reps 2 --arms "" "potrf_mode=2,potrf_lazy=8" "potrf_mode=2,potrf_lazy=4" "potrf_mode=2,potrf_lazy=6" > gpurun_out/stag_16384.log 2>&1 || exit $?
timeout -k 10 150 python3 tools/opt_ab.py --n 8192 --rounds 3 --reps 3 --arms "" "potrf_mode=2,potrf_lazy=2" "potrf_mode=2,potrf_lazy=4" "potrf_mode=2,potrf_lazy=6" > gpurun_out/stag_8192.log 2>&1 || exit $?
timeout -k 10 150 python3 tools/opt_ab.py --n 4096 --batch 4 --rounds 4 --reps 5 --arms "" "potrf_mode=2,potrf_lazy=2" "potrf_mode=2,potrf_lazy=4" "potrf_mode=2,potrf_lazy=6" > gpurun_out/stag_b4.log 2>&1 || exit $?
