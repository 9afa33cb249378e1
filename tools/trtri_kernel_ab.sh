# Times of the triangular inverse at n = 16384 for several libgpx builds (tools/trtri_prof.py, 4 reps per process,
# alternating, two processes each).  Arguments: name=path (relative to the repo root; "name=" = the working tree's).
#   bash tools/trtri_kernel_ab.sh base=ab/libgpx_base.so new=
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out || exit 1
export TMPDIR=/tmp
for i in 1 2; do
  for arm in "$@"; do
    name=${arm%%=*}; lib=${arm#*=}
    if [ -n "$lib" ]; then export GPX_LIB=$PWD/$lib; else unset GPX_LIB; fi
    timeout -k 10 200 python3 tools/trtri_prof.py --n 16384 --reps 4 > gpurun_out/trtri_ab_${name}_$i.log 2>&1 || exit $?
  done
done
unset GPX_LIB
for f in gpurun_out/trtri_ab_*_*.log; do echo "$f $(grep -h 'trtri [0-9]' $f | tr '\n' ' ')"; done
echo TRTRI KERNEL AB DONE
