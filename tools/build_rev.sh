#!/bin/bash
# Build libgpx.so from a git revision's csrc/ + include/ into ab/libgpx_<name>.so (for tools/ab_libs.py A/B runs).
#   tools/build_rev.sh <rev> <name>
set -e
rev=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d /tmp/gpxrev.XXXX)
git -C "$root" archive "$rev" bayesianoptimizer_amd/csrc include | tar -x -C "$tmp"
mkdir -p "$root/ab"
make -C "$tmp/bayesianoptimizer_amd/csrc" -j8 OUT="$root/ab/libgpx_$name.so" OBJDIR="$tmp/obj" > "$tmp/build.log" 2>&1 || { tail -20 "$tmp/build.log"; exit 1; }
rm -rf "$tmp"
echo "built ab/libgpx_$name.so from $rev"
