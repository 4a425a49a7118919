#!/bin/bash
# Shard-balance A/B: the default bench line (no configs, PMC or CPU baseline)
# per variant, REPS rounds; prints value, full-frame ms and the 2/4/8-way
# predictions, shard sums and balance.
#   tools/bal_ab.sh "label:ENV=v,ENV2=w:libdir" ...   (env may be empty, libdir defaults to lib)
set -o pipefail
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do for spec in "$@"; do
IFS=: read -r n envs l <<< "$spec"
envcmd=(env RTGPU_LIB_DIR=${l:-lib})
if [ -n "$envs" ]; then IFS=, read -ra kv <<< "$envs"; envcmd+=("${kv[@]}"); fi
"${envcmd[@]}" timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs --no-pmc --no-three-pass --no-count > gpurun_out/bal_${n}_$rep.json 2> gpurun_out/bal_${n}_$rep.err || { tail -20 gpurun_out/bal_${n}_$rep.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bal_${n}_$rep.json').read().strip().splitlines()[-1]); b=d['shard_balance']
print('$n', d['value'], b['full_frame_ms'], [(k, b[k]['predicted_speedup'], round(sum(b[k]['shard_ms']),1), b[k]['max_over_mean']) for k in ('n2','n4','n8')], flush=True)"
done; done
