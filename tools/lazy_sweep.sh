# potrf lazy-flush sweep (GPX_POTRF_LAZY) at n = 4096, 8192, 16384 (tools/fit_timing.py)
for g in 1 2; do
  GPX_POTRF_LAZY=$g timeout -k 10 60 python tools/fit_timing.py --n 4096 --kernel rbf --reps 5 2>/dev/null | head -1 | sed "s/^/lazy=$g /" || exit 1
done
for g in 1 2 4; do
  GPX_POTRF_LAZY=$g timeout -k 10 60 python tools/fit_timing.py --n 8192 --kernel rbf --reps 3 2>/dev/null | head -1 | sed "s/^/lazy=$g /" || exit 1
done
for g in 4 6 8; do
  GPX_POTRF_LAZY=$g timeout -k 10 120 python tools/fit_timing.py --n 16384 --kernel matern52 --reps 2 2>/dev/null | head -1 | sed "s/^/lazy=$g /" || exit 1
done
