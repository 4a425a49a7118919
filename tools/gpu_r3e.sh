#!/bin/bash
# Round-3 GPU call: GPU suite (tight instance boxes, 4-wave k_shade, twin
# streams), C4 A/B with the shard balance (round-2 HEAD / k_shade 4 waves
# only / this build) and the C2/C3/C5 configs of this build, then (last) the
# RTG_GUARD C3 diagnostic with the device-side bad-index record.
set -o pipefail
mkdir -p gpurun_out/r3e gpurun_out/guard
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3e/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3e/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3e/gpu_tests.log
for rep in 1 2; do
  for lib in lib_head lib_sw4 lib; do
    RTGPU_LIB_DIR=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-count \
      --no-configs --no-three-pass > gpurun_out/r3e/ab_$lib.$rep.json 2> gpurun_out/r3e/ab_$lib.$rep.err \
      || { echo "bench $lib failed"; tail -20 gpurun_out/r3e/ab_$lib.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); b=d['shard_balance']; print(sys.argv[2], d['value'], d['config']['frame_sum'], 'n8', b['n8']['predicted_speedup'])" \
      gpurun_out/r3e/ab_$lib.$rep.json $lib
  done
done
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-count --no-balance --no-three-pass \
  > gpurun_out/r3e/cfg.json 2> gpurun_out/r3e/cfg.err || { echo "cfg failed"; tail -20 gpurun_out/r3e/cfg.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3e/cfg.json')); print({k: (v['value'], v['frame_sum']) for k, v in d['configs'].items()})"
echo r3e-ab-done
RTGPU_LIB_DIR=lib_guard3 timeout -k 10 300 python3 -u tools/guard_diag.py gpurun_out/guard/lib_guard3 \
  > gpurun_out/guard/lib_guard3.log 2>&1 || { echo "diag lib_guard3 failed"; tail -20 gpurun_out/guard/lib_guard3.log; exit 1; }
grep RTG_GUARD gpurun_out/guard/lib_guard3.log | head -5
RTGPU_LIB_DIR=lib timeout -k 10 300 python3 -u tools/guard_diag.py gpurun_out/guard/lib > gpurun_out/guard/lib.log 2>&1 \
  || { echo "diag lib failed"; tail -20 gpurun_out/guard/lib.log; exit 1; }
echo r3e-done
