# sweep chunk size (K* bytes per chunk) re-measured with the groups-of-64 sweep product order (experiment library)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export GPX_LIB=$R/ab/libgpx_xchunk.so
timeout -k 10 700 python3 tools/env_ab.py --rounds 3 --timeout 240 --regex '"value": ([0-9.e+]+)' --regex '"roofline": {[^}]*"frac": ([0-9.]+)' --arms "c512:GPX_X_CHUNK_MIB=512" "c1024:GPX_X_CHUNK_MIB=1024" "c2048:GPX_X_CHUNK_MIB=2048" "c4096:GPX_X_CHUNK_MIB=4096" -- python3 bench.py --steps 5 --warmup 2 --no-other-configs --no-cpu-baseline > gpurun_out/chunk_ab.log 2>&1 || exit $?
