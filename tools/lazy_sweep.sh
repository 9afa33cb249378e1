# potrf schedule sweep: mode 0 (panels apply pending columns), mode 1 (lookahead column + lazy bulk flush),
# mode 2 (lookahead + staggered bulk flush); flush period g (GPX_POTRF_LAZY); tools/fit_timing.py
run() { GPX_OPTIONS=potrf_mode=$1,potrf_lazy=$2 timeout -k 10 120 python tools/fit_timing.py --n $3 --kernel $4 --reps $5 > /tmp/ft.log 2>&1 || return 1; grep "fit:" /tmp/ft.log | sed "s/^/mode=$1 lazy=$2 /"; }
run 0 1 4096 rbf 5 && run 2 1 4096 rbf 5 && run 2 2 4096 rbf 5 && run 2 3 4096 rbf 5 && run 2 4 4096 rbf 5 &&
run 1 4 8192 rbf 3 && run 2 2 8192 rbf 3 && run 2 4 8192 rbf 3 &&
run 1 8 16384 matern52 2 && run 2 4 16384 matern52 2 && run 2 8 16384 matern52 2
