#!/bin/bash
# Round 5: LDS node cache defaults (k_extend 4 nodes + kept 1/d, k_shadow 48)
# against lib_base, the node
# cache read through flat loads (lib_fl); then WRITE_SIZE passes of lib, of a
# build without the result stores (lib_nrs, wrong frames: bounds the stores'
# share) and of the traversal kernels at 6 waves without VGPR spills (lib_w6s).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=${REPS:-2} tools/ab.sh "base::lib_base" "lds::lib" "fl::lib_fl" "w6s::lib_w6s" 2>&1 | tee gpurun_out/r5_lds5_ab.log || exit 1
for v in lib lib_nrs lib_w6s; do
  OUTD=gpurun_out/r5wr_$v
  rm -rf $OUTD; mkdir -p $OUTD
  RTGPU_LIB_DIR=$v RTGPU_STREAMS=1 timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUTD/WRITE_SIZE -o p -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count --no-configs --no-balance --no-three-pass --no-pmc \
    > $OUTD/w.json 2> $OUTD/w.err || exit 1
done
echo done
