#!/bin/bash
# Interleaved A/B of bench.py variants in one GPU call (REPS rounds):
#   tools/ab.sh "label:ENV=v,ENV2=w:libdir[:bench args]" ...      [BENCH_ARGS=..., REPS=2]
# env part may be empty ("a::lib_x"), libdir defaults to lib.  Prints one
# line per run: value, per-kernel ms and the instrumented work per sample.
set -o pipefail
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for spec in "$@"; do
    IFS=: read -r label envs lib vargs <<< "$spec"
    lib=${lib:-lib}
    tag=${label}_$rep
    envcmd=(env RTGPU_LIB_DIR=$lib)
    if [ -n "$envs" ]; then IFS=, read -ra kv <<< "$envs"; envcmd+=("${kv[@]}"); fi
    "${envcmd[@]}" timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs --no-balance \
      $BENCH_ARGS $vargs > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { tail -20 gpurun_out/ab_$tag.err; exit 1; }
    python3 - "$tag" <<'PY'
import json, sys
tag = sys.argv[1]
d = json.loads(open(f"gpurun_out/ab_{tag}.json").read().strip().splitlines()[-1])
w = d.get("work_per_sample") or {}
k = d.get("kernels") or {}
print(tag, d["value"], d["config"].get("nodes"), d["config"].get("frame_sum"), {n: v["ms_total"] for n, v in k.items()},
      {n: w.get(n) for n in ("node_visits", "tri_tests", "quad_tests", "instance_visits", "stack_spills") if n in w},
      flush=True)
PY
  done
done
