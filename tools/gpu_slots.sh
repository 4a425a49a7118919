#!/bin/bash
# Batch-size sweep (path slots per batch, RTGPU_SLOTS) on the default bench workload.
set -o pipefail
mkdir -p gpurun_out
for s in "$@"; do
  RTGPU_SLOTS=$s timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/slots_$s.json 2> gpurun_out/slots_$s.err || { tail -5 gpurun_out/slots_$s.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/slots_$s.json'));print('slots=$s',d['value'],d['roofline']['frac'],{k:v['ms_total'] for k,v in d['kernels'].items()})"
done
