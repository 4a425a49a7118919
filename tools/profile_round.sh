#!/bin/bash
# Round profile of the default bench workload (one gpurun call):
#   1. rocprofv3 --kernel-trace --stats of bench.py on one stream
#      (RTGPU_STREAMS=1, the single-stream attribution the bench line uses)
#   2. separate --pmc passes for FETCH_SIZE and WRITE_SIZE (HBM traffic),
#      never combined with tracing, on the same workload (500 spp, one step:
#      the same per-launch batches as the timed bench steps)
# Outputs under gpurun_out/prof/ (OUT=...); tools/pmc_traffic.py turns them
# into profiles/pmc_<scene>_<W>x<H>.json.  SCENE_ARGS selects another
# workload, e.g. SCENE_ARGS="--scene cornell --width 600 --aspect 1 --spp 1000" (C3).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
mkdir -p $OUT
RTGPU_STREAMS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs --no-balance --no-pmc --no-three-pass $SCENE_ARGS > $OUT/kt_bench.json 2> $OUT/kt.err || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  RTGPU_STREAMS=1 timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o p -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count --no-configs --no-balance --no-three-pass $SCENE_ARGS > $OUT/$c.json 2> $OUT/$c.err || exit 1
done
echo done
