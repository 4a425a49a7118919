#!/bin/bash
# GPU tests on the default build, then one BASELINE config benched on several
# in-tree builds, two rounds:  tools/gpu_cfg_ab.sh "<bench args>" lib lib_x ...
set -o pipefail
mkdir -p gpurun_out
args=$1; shift
libs=("$@")
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cfgab_tests.log 2>&1 || { tail -30 gpurun_out/cfgab_tests.log; exit 1; }
tail -1 gpurun_out/cfgab_tests.log
for rep in 1 2; do
  for lib in "${libs[@]}"; do
    RTGPU_LIB_DIR=$lib timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs --no-balance $args > gpurun_out/cfgab.json 2> gpurun_out/cfgab.err || { tail -20 gpurun_out/cfgab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/cfgab.json'));k=d.get('kernels',{});print('$lib',d['value'],repr(d['config']['frame_sum']),{n:v['ms_avg'] for n,v in k.items()})"
  done
done
