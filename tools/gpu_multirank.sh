#!/bin/bash
# Rehearse bench.py's multi-rank path on a one-GPU box: N ranks share the
# GPU, gloo carries the reduce; the frame checksum must equal the N=1 run.
set -o pipefail
mkdir -p gpurun_out
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-count --no-configs --no-balance --spp ${SPP:-64}"
timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/mr_1.json 2> gpurun_out/mr_1.err || { tail -20 gpurun_out/mr_1.err; exit 1; }
for n in 2 4; do
  RTGPU_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n $ARGS > gpurun_out/mr_$n.json 2> gpurun_out/mr_$n.err || { tail -20 gpurun_out/mr_$n.err; exit 1; }
done
python3 - <<'PY'
import json
r = {n: json.loads(open(f"gpurun_out/mr_{n}.json").read().strip().splitlines()[-1]) for n in (1, 2, 4)}
for n, d in r.items():
    print(n, d["n_gpus"], d["value"], d["ms_per_step"], d["config"]["parallelism"], d["config"]["frame_sum"])
assert all(d["config"]["frame_sum"] == r[1]["config"]["frame_sum"] for d in r.values()), "frame checksum differs"
print("multirank-ok")
PY
