# Schedule re-tune after the hand-placed trailing tiles (every schedule gives the same bits: opt_ab checks alpha).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u tools/opt_ab.py --n 4096 --rounds 5 --reps 10 --arms "" "potrf_switch=0" "potrf_switch=5" "potrf_switch=13" "potrf_switch=17" "potrf_switch=25" "potrf_switch=9,potrf_lazy=2" "potrf_switch=13,potrf_lazy=6" "potrf_switch=17,potrf_lazy=8" > gpurun_out/r05_sched_4096.log 2>&1 &&
timeout -k 10 400 python -u tools/opt_ab.py --n 4096 --batch 4 --rounds 4 --reps 5 --arms "" "potrf_lazy=4" "potrf_lazy=8" "potrf_switch=25" "potrf_switch=37" "potrf_switch=49" > gpurun_out/r05_sched_4096_b4.log 2>&1 &&
timeout -k 10 500 python -u tools/opt_ab.py --n 16384 --kernel matern52 --rounds 2 --reps 2 --arms "" "potrf_lazy=6" "potrf_lazy=12" "potrf_lazy=8,potrf_switch=193" "potrf_lazy=8,potrf_switch=225" > gpurun_out/r05_sched_16384.log 2>&1 &&
timeout -k 10 300 python -u tools/opt_ab.py --n 8192 --rounds 3 --reps 3 --arms "" "potrf_lazy=4" "potrf_lazy=8" "potrf_lazy=6,potrf_switch=67" > gpurun_out/r05_sched_8192.log 2>&1
