#!/bin/bash
# Round-3 GPU call: no-prefetch tail A/B (C4 value + 8-way shard prediction),
# and the kernel-trace anatomy of a twin-stream 1/8 shard.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3f
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3f/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3f/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3f/gpu_tests.log
for rep in 1 2; do
  for lib in lib_pf lib; do
    RTGPU_LIB_DIR=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-count \
      --no-configs --no-three-pass > gpurun_out/r3f/ab_$lib.$rep.json 2> gpurun_out/r3f/ab_$lib.$rep.err \
      || { echo "bench $lib failed"; tail -20 gpurun_out/r3f/ab_$lib.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); b=d['shard_balance']; print(sys.argv[2], d['value'], d['config']['frame_sum'], 'n8', b['n8']['predicted_speedup'], max(b['n8']['shard_device_ms']))" \
      gpurun_out/r3f/ab_$lib.$rep.json $lib
  done
done
RTGPU_STREAMS=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3f/sp2 -o kt -- \
  python3 tools/shard_probe.py > gpurun_out/r3f/sp2.log 2>&1 || { echo "shard probe failed"; tail -20 gpurun_out/r3f/sp2.log; exit 1; }
python3 tools/shard_probe.py --analyze gpurun_out/r3f/sp2 > gpurun_out/r3f/sp2_analysis.txt 2>&1
grep render gpurun_out/r3f/sp2_analysis.txt
echo r3f-done
