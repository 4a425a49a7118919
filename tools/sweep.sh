#!/bin/bash
# quick A/B of runtime knobs on a reduced Lucy frame
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-count --spp 100"
for r in 4 8 16 32 48; do
  echo -n "refill=$r "; RTGPU_REFILL=$r timeout -k 10 120 python bench.py $ARGS 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
