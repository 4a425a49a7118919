#!/bin/bash
# Round 3: GPU suite on the lean-shade / auto-twin build, then A/B on C4:
# auto twins (one stream at full frame) vs forced twins vs the 64-B triangle
# shading record (lib_tris); full lines (PMC, balance) then quick repeats.
set -o pipefail
OUT=gpurun_out/r3ab2
mkdir -p $OUT
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
run() {
  name=$1; lib=$2; streams=$3; shift 3
  RTGPU_STREAMS=$streams RTGPU_LIB_DIR=$lib timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    --no-configs --no-three-pass "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -20 $OUT/$name.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; b=d.get('shard_balance') or {}
print(sys.argv[2], d['value'], d['config']['frame_sum'], 'frac', r.get('frac'), 'n8', (b.get('n8') or {}).get('predicted_speedup'),
      {k: (v['ms_avg'], v.get('hbm_frac'), v.get('l2_served'), v.get('twins')) for k, v in (d.get('kernels') or {}).items()})" $OUT/$name.json $name
}
run auto lib 0 || exit 1
run twins lib 2 || exit 1
run tris lib_tris 0 || exit 1
for rep in 2 3; do
  run auto.q$rep lib 0 --no-pmc --no-balance --no-count || exit 1
  run tris.q$rep lib_tris 0 --no-pmc --no-balance --no-count || exit 1
  run twins.q$rep lib 2 --no-pmc --no-balance --no-count || exit 1
done
echo ab2-done
