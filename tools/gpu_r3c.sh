#!/bin/bash
# Round-3 GPU call: GPU suite on the twin-stream build, C4 A/B (round-2 HEAD,
# this build with 1 and 2 streams), the shard balance, then (last, it may
# fault) the RTG_GUARD C3 diagnostic with per-launch fault attribution.
set -o pipefail
mkdir -p gpurun_out/r3c gpurun_out/guard
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3c/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3c/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3c/gpu_tests.log
for rep in 1 2; do
  for v in head:lib_head:2 s1:lib:1 s2:lib:2; do
    IFS=: read name lib streams <<< "$v"
    RTGPU_STREAMS=$streams RTGPU_LIB_DIR=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline \
      --no-count --no-configs --no-three-pass > gpurun_out/r3c/ab_$name.$rep.json 2> gpurun_out/r3c/ab_$name.$rep.err \
      || { echo "bench $name failed"; tail -20 gpurun_out/r3c/ab_$name.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); b=d['shard_balance']; print(sys.argv[2], d['value'], d['config']['frame_sum'], 'n8', b['n8']['predicted_speedup'], max(b['n8']['shard_device_ms']))" \
      gpurun_out/r3c/ab_$name.$rep.json $name
  done
done
echo r3c-ab-done
RTGPU_DEBUG_SYNC=1 RTGPU_LIB_DIR=lib_guard2 timeout -k 10 300 python3 -u tools/guard_diag.py gpurun_out/guard/lib_guard2 \
  > gpurun_out/guard/lib_guard2.log 2>&1 || { echo "diag lib_guard2 failed"; tail -20 gpurun_out/guard/lib_guard2.log; exit 1; }
grep -c RTG_GUARD gpurun_out/guard/lib_guard2.log
echo r3c-done
