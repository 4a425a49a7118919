#!/bin/bash
# Round-3 first GPU call: GPU suite on the new build (schedule-independence
# test included), the RTG_GUARD C3 diagnostic renders (guard vs HEAD
# production), and a C4 A/B of the traversal variants.
set -o pipefail
mkdir -p gpurun_out/r3a gpurun_out/guard
[ -f gpurun_out/r3a/avail.txt ] || (cd /tmp && TMPDIR=/tmp timeout -k 10 90 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/r3a/avail.txt 2>&1) || echo "list-avail failed"
[ -n "$R3A_SKIP_TESTS" ] || timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3a/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3a/gpu_tests.log; exit 1; }
[ -n "$R3A_SKIP_TESTS" ] || tail -2 gpurun_out/r3a/gpu_tests.log
if [ -n "$R3A_GUARD" ]; then
for lib in lib_guard lib_head lib; do
  RTGPU_LIB_DIR=$lib timeout -k 10 200 python3 -u tools/guard_diag.py gpurun_out/guard/$lib \
    > gpurun_out/guard/$lib.log 2>&1 || { echo "diag $lib failed"; tail -20 gpurun_out/guard/$lib.log; exit 1; }
  grep -c RTG_GUARD gpurun_out/guard/$lib.log
done
fi
for rep in 1 2; do
  for lib in lib_head lib lib_spec lib_nowiden; do
    RTGPU_LIB_DIR=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-count \
      --no-configs --no-balance --no-three-pass > gpurun_out/r3a/ab_$lib.$rep.json 2> gpurun_out/r3a/ab_$lib.$rep.err \
      || { echo "bench $lib failed"; tail -20 gpurun_out/r3a/ab_$lib.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'])" \
      gpurun_out/r3a/ab_$lib.$rep.json $lib
  done
done
echo r3a-ab-done
# live PMC passes inside bench.py (default run minus the configs / balance legs)
timeout -k 10 500 python3 bench.py --no-configs --no-balance --cpu-spp 8 > gpurun_out/r3a/bench_pmc.json 2> gpurun_out/r3a/bench_pmc.err \
  || { echo "bench pmc failed"; tail -20 gpurun_out/r3a/bench_pmc.err; exit 1; }
cat gpurun_out/r3a/bench_pmc.json
echo r3a-pmc-done
