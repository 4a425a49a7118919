#!/bin/bash
# single-stream kernel traces of C2 and C5 (one step each)
export TMPDIR=/tmp
mkdir -p gpurun_out/r05_trace
for sc in "random 1200 500" "hdri-test 1920 2000"; do
  set -- $sc
  RTGPU_STREAMS=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05_trace/$1 -o t -- \
    python3 bench.py --scene $1 --width $2 --spp $3 --steps 1 --warmup 1 --no-pmc --no-cpu-baseline --no-count --no-configs --no-balance --no-three-pass > gpurun_out/r05_trace/$1.json 2> gpurun_out/r05_trace/$1.err || exit 1
done
