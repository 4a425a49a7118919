#!/bin/bash
# A/B of the k_shade octant-ordered survivor output (lib_oct) and the lean
# shade variant (lib_lean: no Noise / Image texture code) against the
# production build on C4 (value, per-kernel ms, frame checksum), two rounds.
set -o pipefail
OUT=gpurun_out/r3oct
mkdir -p $OUT
for rep in 1 2; do
  for v in base:lib oct:lib_oct lean:lib_lean lean5:lib_lean5; do
    IFS=: read name lib <<< "$v"
    RTGPU_LIB_DIR=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline \
      --no-count --no-configs --no-three-pass --no-balance > $OUT/ab_$name.$rep.json 2> $OUT/ab_$name.$rep.err \
      || { echo "bench $name failed"; tail -20 $OUT/ab_$name.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'], {k: (v['ms_avg'], v.get('l2_hit'), v.get('valu_lane_util')) for k, v in d['kernels'].items()})" \
      $OUT/ab_$name.$rep.json $name
  done
done
echo ab-oct-done
