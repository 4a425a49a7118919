#!/bin/bash
# Interleaved short C4 benches of (build, env) variants, two rounds:
#   tools/gpu_sweep.sh "lib RTGPU_REFILL=16" "lib_x RTGPU_REFILL=8" ...
set -o pipefail
mkdir -p gpurun_out
variants=("$@")
for rep in 1 2; do
  for v in "${variants[@]}"; do
    read -r lib envs <<< "$v"
    env RTGPU_LIB_DIR=$lib $envs timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs --no-balance --no-count > gpurun_out/sweep.json 2> gpurun_out/sweep.err || { tail -20 gpurun_out/sweep.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/sweep.json'));print('$v',d['value'],repr(d['config']['frame_sum']))"
  done
done
