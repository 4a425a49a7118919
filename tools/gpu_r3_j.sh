#!/bin/bash
# Round 3: C4 with the automatic twin count (3 at full frame), then the
# persistent traversal grids capped (RTGPU_MAX_BLOCKS; full = 7 x 256 CUs =
# 1792 blocks) so that the twins' kernels share the CUs throughout.
set -o pipefail
OUT=gpurun_out/r3j
mkdir -p $OUT
b() {   # name maxblocks
  RTGPU_MAX_BLOCKS=$2 timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs \
    --no-three-pass --no-pmc --no-count $3 > $OUT/$1.json 2> $OUT/$1.err || { echo "bench $1 failed"; tail -20 $OUT/$1.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); b=d.get('shard_balance') or {}; print(sys.argv[2], d['value'], d['config']['frame_sum'], 'n8', (b.get('n8') or {}).get('predicted_speedup'))" $OUT/$1.json $1
}
b auto.1 0 || exit 1
for rep in 1 2; do
  b cap0.$rep 0 --no-balance || exit 1
  b cap1344.$rep 1344 --no-balance || exit 1
  b cap1024.$rep 1024 --no-balance || exit 1
done
echo r3j-done
