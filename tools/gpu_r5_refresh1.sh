#!/bin/bash
# Round-5 refresh, part 1: GPU tests, smoke, fp64 tolerance, bench line,
# kernel trace + HBM traffic passes (tools/profile_round.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -k "fp64 or three_passes" -q -s --timeout 120 --timeout-method thread > gpurun_out/fp64_tolerance.log 2>&1 || { tail -30 gpurun_out/fp64_tolerance.log; exit 1; }
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
bash tools/profile_round.sh || exit 1
echo refresh1-done
