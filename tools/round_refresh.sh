#!/bin/bash
# Round-end refresh on one GPU box: GPU tests, the default bench line (with
# the CPU baseline), the rocprof kernel-trace + PMC traffic passes, the PMC
# counter passes and one bench line per BASELINE config.  Every GPU step has
# its own time limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
# the fp32-vs-fp64 tolerance figures per BASELINE config (printed by the test)
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -k "fp64 or three_passes" -q -s --timeout 120 --timeout-method thread > gpurun_out/fp64_tolerance.log 2>&1 || { tail -30 gpurun_out/fp64_tolerance.log; exit 1; }
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
bash tools/profile_round.sh || exit 1
bash tools/pmc_profile.sh || exit 1
bash tools/configs_round.sh || exit 1
echo refresh-done
