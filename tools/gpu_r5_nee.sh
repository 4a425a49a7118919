#!/bin/bash
# Round 5: k_nee_apply reading the job's contribution with its visibility word (lib_ne) against the default; kernel trace for the apply times.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=${REPS:-2} bash tools/ab.sh "def::lib" "ne::lib_ne" 2>&1 | tee gpurun_out/r5_nee_ab.log || exit 1
for v in lib lib_ne; do
  RTGPU_LIB_DIR=$v RTGPU_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nee_$v -o kt -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count --no-configs --no-balance --no-pmc --no-three-pass > gpurun_out/nee_$v.json 2>&1 || exit 1
  grep nee_apply gpurun_out/nee_$v/kt_kernel_stats.csv | cut -d, -f2-4
done
