#!/bin/bash
# Round-3 GPU call: GPU suite on the XCD-segmented claim pools, A/B against
# the same build without segments (C4 value + 8-way shard prediction), live
# PMC line of the segmented build (L2 hit rate).
set -o pipefail
mkdir -p gpurun_out/r3g
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3g/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3g/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3g/gpu_tests.log
for rep in 1 2; do
  for lib in lib_noseg lib; do
    RTGPU_LIB_DIR=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-count \
      --no-configs --no-three-pass > gpurun_out/r3g/ab_$lib.$rep.json 2> gpurun_out/r3g/ab_$lib.$rep.err \
      || { echo "bench $lib failed"; tail -20 gpurun_out/r3g/ab_$lib.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); b=d['shard_balance']; print(sys.argv[2], d['value'], d['config']['frame_sum'], 'n8', b['n8']['predicted_speedup'], max(b['n8']['shard_device_ms']))" \
      gpurun_out/r3g/ab_$lib.$rep.json $lib
  done
done
for lib in lib_noseg lib; do
  RTGPU_LIB_DIR=$lib timeout -k 10 400 python3 bench.py --no-configs --no-balance --no-three-pass --no-cpu-baseline \
    > gpurun_out/r3g/pmc_$lib.json 2> gpurun_out/r3g/pmc_$lib.err || { echo "pmc $lib failed"; tail -20 gpurun_out/r3g/pmc_$lib.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['kernels']; print(sys.argv[2], {k: (v['ms_avg'], v.get('l2_hit'), v.get('hbm_frac'), v.get('l2_read_latency_cycles')) for k, v in d.items()})" \
    gpurun_out/r3g/pmc_$lib.json $lib
done
echo r3g-done
