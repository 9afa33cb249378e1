# A/B of the panel split policy (GPX_OPT_POTRF_SPLIT) on the update at n = 16384 / 8192 / 4096 and B = 4 x 4096,
# plus the new invalid-argument test
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_outputs.py::test_per_output_entry_points_reject_invalid_arguments > gpurun_out/ab/invalid.log 2>&1 &&
timeout -k 10 300 python3 -u tools/opt_ab.py --n 16384 --kernel matern52 --rounds 3 --reps 3 --arms "" "potrf_split=3" "potrf_split=1" > gpurun_out/ab/split_16384.log 2>&1 &&
timeout -k 10 200 python3 -u tools/opt_ab.py --n 8192 --rounds 5 --reps 8 --arms "" "potrf_split=3" "potrf_split=1" > gpurun_out/ab/split_8192.log 2>&1 &&
timeout -k 10 200 python3 -u tools/opt_ab.py --n 4096 --rounds 7 --reps 20 --arms "" "potrf_split=3" "potrf_split=1" > gpurun_out/ab/split_4096.log 2>&1 &&
timeout -k 10 200 python3 -u tools/opt_ab.py --n 4096 --batch 4 --rounds 5 --reps 10 --arms "" "potrf_split=3" "potrf_split=1" > gpurun_out/ab/split_b4.log 2>&1
rc=$?
tail -2 gpurun_out/ab/invalid.log; for f in split_16384 split_8192 split_4096 split_b4; do echo == $f; tail -5 gpurun_out/ab/$f.log; done
exit $rc
