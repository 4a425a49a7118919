#!/bin/bash
# Round 3: refresh (parts a and b) of the final build, then C4 A/B of
# k_shadow at 6 waves per SIMD (lib_sw6: 79 VGPRs, no spills) against 7.
set -o pipefail
bash tools/gpu_r3_final.sh a || exit 1
bash tools/gpu_r3_final.sh b || exit 1
OUT=gpurun_out/r3l
mkdir -p $OUT
for rep in 1 2; do
  for v in base:lib sw6:lib_sw6; do
    IFS=: read name lib <<< "$v"
    RTGPU_LIB_DIR=$lib timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
      --no-pmc --no-balance > $OUT/$name.$rep.json 2> $OUT/$name.$rep.err || { echo "bench $name failed"; tail -20 $OUT/$name.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'], {k: v['ms_avg'] for k, v in d['kernels'].items()})" $OUT/$name.$rep.json $name.$rep
  done
done
echo r3l-done
