# Fused small-n sweep: GPU parity (fused vs oracle vs unfused) and candidates/s with the fused path on and off.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_small_n.py -x -v --timeout 120 --timeout-method thread > gpurun_out/small_n_tests.log 2>&1 &&
timeout -k 10 120 python -u tools/small_n_rates.py 64 128 256 > gpurun_out/small_rates_fused.log 2>&1 &&
timeout -k 10 120 python -u tools/small_n_posterior_rates.py > gpurun_out/small_post_fused.log 2>&1 &&
GPX_OPTIONS=sweep_fused=0 timeout -k 10 120 python -u tools/small_n_posterior_rates.py > gpurun_out/small_post_unfused.log 2>&1
