# batched (B = 4, n = 4096) schedule sweep around the default (lookahead g = 6, eager from ~49)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python3 tools/opt_ab.py --n 4096 --batch 4 --rounds 4 --reps 5 --arms "" "potrf_lazy=6,potrf_mode=1,potrf_switch=55" "potrf_lazy=6,potrf_mode=1,potrf_switch=43" "potrf_lazy=5,potrf_mode=1,potrf_switch=51" "potrf_lazy=7,potrf_mode=1,potrf_switch=50" "potrf_lazy=8,potrf_mode=1,potrf_switch=49" "potrf_lazy=4,potrf_mode=1,potrf_switch=49" "potrf_lazy=3,potrf_mode=1,potrf_switch=49" > gpurun_out/b4_sched.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/opt_ab.py --n 4096 --batch 2 --rounds 4 --reps 5 --arms "" "potrf_lazy=4,potrf_mode=1,potrf_switch=49" "potrf_lazy=6,potrf_mode=1,potrf_switch=49" "potrf_lazy=4,potrf_mode=1,potrf_switch=41" > gpurun_out/b2_sched.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/opt_ab.py --n 4096 --batch 8 --rounds 3 --reps 3 --arms "" "potrf_lazy=6,potrf_mode=1,potrf_switch=55" "potrf_lazy=8,potrf_mode=1,potrf_switch=49" "potrf_lazy=6,potrf_mode=1,potrf_switch=37" > gpurun_out/b8_sched.log 2>&1 || exit $?
