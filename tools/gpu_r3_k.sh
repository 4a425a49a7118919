#!/bin/bash
# Round 3: refresh part b (profiles) of the current build, then C4 A/B of the
# inlined slow-camera path (lib_isc: fewer VGPR spills in the bounce-0
# kernels) against the production build.
set -o pipefail
bash tools/gpu_r3_final.sh b || exit 1
OUT=gpurun_out/r3k
mkdir -p $OUT
for rep in 1 2; do
  for v in base:lib isc:lib_isc; do
    IFS=: read name lib <<< "$v"
    RTGPU_LIB_DIR=$lib timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
      --no-pmc --no-balance > $OUT/$name.$rep.json 2> $OUT/$name.$rep.err || { echo "bench $name failed"; tail -20 $OUT/$name.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'], {k: v['ms_avg'] for k, v in d['kernels'].items()})" $OUT/$name.$rep.json $name.$rep
  done
done
echo r3k-done
