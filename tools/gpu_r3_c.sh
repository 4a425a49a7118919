#!/bin/bash
# Round 3: GPU suite + fp64 tolerance + default bench line on the current
# build, A/B of temporal hit-record stores (lib_hitt), then the rocprof
# kernel-trace / FETCH / WRITE passes of the single-stream attribution.
set -o pipefail
OUT=gpurun_out/r3c
mkdir -p $OUT
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 240 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -k "fp64 or three_passes" -q -s --timeout 120 --timeout-method thread > $OUT/fp64_tolerance.log 2>&1 || { tail -30 $OUT/fp64_tolerance.log; exit 1; }
timeout -k 10 480 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; b=d['shard_balance']
print('bench', d['value'], d['config']['frame_sum'], 'frac', r['frac'], 'n8', b['n8']['predicted_speedup'], {k: v for k, v in d['configs'].items()})
print({k: (v['ms_avg'], v.get('hbm_frac'), v.get('l2_served'), v.get('twins')) for k, v in d['kernels'].items()})" $OUT/bench.json
for rep in 1 2; do
  for v in base:lib hitt:lib_hitt; do
    IFS=: read name lib <<< "$v"
    RTGPU_LIB_DIR=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
      --no-balance --no-pmc --no-count > $OUT/ab_$name.$rep.json 2> $OUT/ab_$name.$rep.err || { echo "ab $name failed"; tail -20 $OUT/ab_$name.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'])" $OUT/ab_$name.$rep.json $name
  done
done
OUT=$OUT/prof bash tools/profile_round.sh || exit 1
echo r3c-done
