#!/bin/bash
# Build the kernels of a git revision into go-raytracing_amd/lib_<name> for an
# in-call A/B on the GPU box (RTGPU_LIB_DIR=lib_<name> selects it):
#   tools/build_variant.sh <rev> <name>
set -euo pipefail
rev=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" go-raytracing_amd/csrc include | tar -x -C "$tmp"
make -s -C "$tmp/go-raytracing_amd/csrc" -j8 OUT="$root/go-raytracing_amd/lib_$name" > /dev/null
rm -rf "$tmp"
echo "built $rev -> go-raytracing_amd/lib_$name"
