#!/bin/bash
# Round 3: C4 A/B of the unrolled k_nee_apply (lib_nee4, 4 jobs per thread
# and iteration) against the production build; kernel split from the
# single-stream attribution (no PMC).
set -o pipefail
OUT=gpurun_out/r3e
mkdir -p $OUT
for rep in 1 2; do
  for v in base:lib nee4:lib_nee4; do
    IFS=: read name lib <<< "$v"
    RTGPU_LIB_DIR=$lib timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
      --no-pmc --no-balance > $OUT/$name.$rep.json 2> $OUT/$name.$rep.err || { echo "bench $name failed"; tail -20 $OUT/$name.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'], {k: v['ms_avg'] for k, v in d['kernels'].items()})" $OUT/$name.$rep.json $name.$rep
  done
done
RTGPU_LIB_DIR=lib_nee4 RTGPU_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_nee4 -o kt -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-configs --no-balance --no-pmc --no-three-pass --no-count > $OUT/kt_nee4.json 2> $OUT/kt_nee4.err || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
echo r3e-done
