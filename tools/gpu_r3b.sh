#!/bin/bash
# Round-3 GPU call: GPU suite, C4 A/B (HEAD of round 2 vs this build), the
# default bench line (live PMC, configs, shard balance, 3-pass reference
# workload, CPU baseline).
set -o pipefail
mkdir -p gpurun_out/r3b
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3b/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3b/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3b/gpu_tests.log
for rep in 1 2; do
  for lib in lib_head lib; do
    RTGPU_LIB_DIR=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-count \
      --no-configs --no-balance --no-three-pass > gpurun_out/r3b/ab_$lib.$rep.json 2> gpurun_out/r3b/ab_$lib.$rep.err \
      || { echo "bench $lib failed"; tail -20 gpurun_out/r3b/ab_$lib.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'])" \
      gpurun_out/r3b/ab_$lib.$rep.json $lib
  done
done
timeout -k 10 600 python3 bench.py > gpurun_out/r3b/bench.json 2> gpurun_out/r3b/bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/r3b/bench.err; exit 1; }
cat gpurun_out/r3b/bench.json
echo r3b-done
