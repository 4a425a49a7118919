#!/bin/bash
# GPU parity suite, then bench under several env settings (one gpurun call).
# usage: tools/gpu_ab2.sh "ENV1=a" "ENV1=b" ...
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || { tail -20 gpurun_out/ab_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$i.json'));print('$e',d['value'],d['roofline']['frac'],{k:v['ms_total'] for k,v in d['kernels'].items()})"
done
