#!/bin/bash
# GPU parity suite + bench A/B of the two BLAS builders (one gpurun call).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for b in reference sah; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --blas $b > gpurun_out/bench_$b.json 2> gpurun_out/bench_$b.err || { tail -20 gpurun_out/bench_$b.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_$b.json'));print('$b',d['value'],d['roofline']['frac'],{k:v['ms_total'] for k,v in d['kernels'].items()},d['work_per_sample'])"
done
