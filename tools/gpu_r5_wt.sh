#!/bin/bash
# Round 5: wave timeline with claim statistics (RTG_WAVETIME build, lib_wt),
# one stream, the shard-anatomy renders (full frame, 1/N shards).
set -o pipefail
mkdir -p gpurun_out
RTGPU_LIB_DIR=lib_wt RTGPU_STREAMS=1 timeout -k 10 500 python3 tools/shard_anat.py > gpurun_out/r5_wt.out 2> gpurun_out/r5_wt.log || { tail -20 gpurun_out/r5_wt.log; exit 1; }
grep -A2 "k_extend b0" gpurun_out/r5_wt.log | head -60
