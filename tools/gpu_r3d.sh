#!/bin/bash
# Round-3 GPU call: kernel-trace anatomy of a full C4 frame vs a 1/8 shard,
# k_shade at 4 waves A/B, then (last, it may fault) the RTG_GUARD C3
# diagnostic of the current code with per-launch fault attribution.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3d gpurun_out/guard
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3d/sp -o kt -- \
  python3 tools/shard_probe.py > gpurun_out/r3d/sp.log 2>&1 || { echo "shard probe failed"; tail -20 gpurun_out/r3d/sp.log; exit 1; }
python3 tools/shard_probe.py --analyze gpurun_out/r3d/sp > gpurun_out/r3d/sp_analysis.txt 2>&1
head -5 gpurun_out/r3d/sp_analysis.txt
for rep in 1 2; do
  for lib in lib lib_sw4; do
    RTGPU_LIB_DIR=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-count \
      --no-configs --no-three-pass --no-balance > gpurun_out/r3d/ab_$lib.$rep.json 2> gpurun_out/r3d/ab_$lib.$rep.err \
      || { echo "bench $lib failed"; tail -20 gpurun_out/r3d/ab_$lib.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'])" \
      gpurun_out/r3d/ab_$lib.$rep.json $lib
  done
done
echo r3d-ab-done
RTGPU_DEBUG_SYNC=1 RTGPU_LIB_DIR=lib_guard2 timeout -k 10 300 python3 -u tools/guard_diag.py gpurun_out/guard/lib_guard2 \
  > gpurun_out/guard/lib_guard2.log 2>&1 || { echo "diag lib_guard2 failed"; tail -20 gpurun_out/guard/lib_guard2.log; exit 1; }
grep -c RTG_GUARD gpurun_out/guard/lib_guard2.log
RTGPU_LIB_DIR=lib timeout -k 10 300 python3 -u tools/guard_diag.py gpurun_out/guard/lib > gpurun_out/guard/lib.log 2>&1 \
  || { echo "diag lib failed"; tail -20 gpurun_out/guard/lib.log; exit 1; }
echo r3d-done
