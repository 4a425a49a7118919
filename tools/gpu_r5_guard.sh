#!/bin/bash
# Round 5: the RTG_GUARD canary build of the LDS-node / claim-order code over
# 1-4 twins and six scenes, then the per-launch anatomy of 1/N shards
# (single stream, kernel trace) on the production build.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
RTGPU_LIB_DIR=lib_guard timeout -k 10 400 python3 tools/guard_sweep.py > gpurun_out/r5_guard_sweep.log 2>&1 || { tail -20 gpurun_out/r5_guard_sweep.log; exit 1; }
tail -5 gpurun_out/r5_guard_sweep.log
RTGPU_STREAMS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sa -o kt -- python3 tools/shard_anat.py > gpurun_out/r5_sa_run.log 2>&1 || { tail -20 gpurun_out/r5_sa_run.log; exit 1; }
python3 tools/shard_anat.py --analyze gpurun_out/sa > gpurun_out/r5_shard_anatomy.txt 2>&1
cat gpurun_out/r5_shard_anatomy.txt
