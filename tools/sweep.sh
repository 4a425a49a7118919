#!/bin/bash
# Throughput sweep of a runtime knob (env var) on the default bench workload.
# usage: tools/sweep.sh VAR v1 v2 ...
VAR=$1; shift
for v in "$@"; do
  env $VAR=$v timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-count > gpurun_out/sweep_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/sweep_$v.json'));print('$VAR=$v',d['value'],d['ms_per_step'])"
done
