#!/bin/bash
# Round-3 GPU call: GPU suite (k_shade chunks per XCD segment), then A/B of
# k_shade segments on/off and of one vs two twin streams (C4 value + 8-way
# shard prediction), then the single-stream live PMC line.
set -o pipefail
mkdir -p gpurun_out/r3h
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3h/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3h/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3h/gpu_tests.log
for rep in 1 2; do
  for v in shnoseg:lib_shnoseg:2 s2:lib:2 s1:lib:1; do
    IFS=: read name lib streams <<< "$v"
    RTGPU_STREAMS=$streams RTGPU_LIB_DIR=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline \
      --no-count --no-configs --no-three-pass > gpurun_out/r3h/ab_$name.$rep.json 2> gpurun_out/r3h/ab_$name.$rep.err \
      || { echo "bench $name failed"; tail -20 gpurun_out/r3h/ab_$name.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); b=d['shard_balance']; print(sys.argv[2], d['value'], d['config']['frame_sum'], 'n8', b['n8']['predicted_speedup'], max(b['n8']['shard_device_ms']))" \
      gpurun_out/r3h/ab_$name.$rep.json $name
  done
done
RTGPU_STREAMS=1 timeout -k 10 400 python3 bench.py --no-configs --no-balance --no-three-pass --no-cpu-baseline \
  > gpurun_out/r3h/pmc_s1.json 2> gpurun_out/r3h/pmc_s1.err || { echo "pmc failed"; tail -20 gpurun_out/r3h/pmc_s1.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline']['frac'], {k: (v['ms_avg'], v.get('l2_hit'), v.get('hbm_frac'), v.get('valu_lane_util')) for k, v in d['kernels'].items()})" gpurun_out/r3h/pmc_s1.json
echo r3h-done
