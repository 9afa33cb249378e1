# potrf schedule sweep: mode 0 (panels apply pending columns) vs mode 1 (lookahead column + lazy bulk flush),
# flush period g (GPX_POTRF_LAZY), at n = 4096, 8192, 16384 (tools/fit_timing.py)
run() { GPX_POTRF_MODE=$1 GPX_POTRF_LAZY=$2 timeout -k 10 120 python tools/fit_timing.py --n $3 --kernel $4 --reps $5 > /tmp/ft.log 2>&1 || return 1; grep "fit:" /tmp/ft.log | sed "s/^/mode=$1 lazy=$2 /"; }
run 0 1 4096 rbf 5 && run 1 1 4096 rbf 5 && run 1 2 4096 rbf 5 && run 1 3 4096 rbf 5 && run 1 4 4096 rbf 5 &&
run 0 2 8192 rbf 3 && run 1 2 8192 rbf 3 && run 1 4 8192 rbf 3 &&
run 0 4 16384 matern52 2 && run 1 4 16384 matern52 2 && run 1 8 16384 matern52 2
