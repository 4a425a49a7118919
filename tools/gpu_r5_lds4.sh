#!/bin/bash
# Round 5: the LDS node cache defaults (lib: k_extend keeps the world 1/d, no
# nodes; k_shadow 48 nodes) against lib_base, k_extend with 4 LDS nodes
# (lib_w4), k_shadow with 52 (lib_s52), temporal result stores (lib_tmp);
# then WRITE_SIZE passes (single stream, one step) of lib and lib_tmp.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=${REPS:-3} tools/ab.sh "base::lib_base" "lds::lib" "w4::lib_w4" "s52::lib_s52" "tmp::lib_tmp" 2>&1 | tee gpurun_out/r5_lds4_ab.log || exit 1
for v in lib lib_tmp; do
  OUTD=gpurun_out/r5wr_$v
  mkdir -p $OUTD
  RTGPU_LIB_DIR=$v RTGPU_STREAMS=1 timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUTD/WRITE_SIZE -o p -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count --no-configs --no-balance --no-three-pass --no-pmc \
    > $OUTD/w.json 2> $OUTD/w.err || exit 1
done
echo done
