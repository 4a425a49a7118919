#!/bin/bash
# Round 5: per-bounce hit / NEE parity of the final build (test_gpu_paths,
# verbose) and the 48-sample full-resolution C4 ray scan.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_paths.py -m gpu -q -s --timeout 300 --timeout-method thread > gpurun_out/r5_path_parity.log 2>&1 || { tail -30 gpurun_out/r5_path_parity.log; exit 1; }
tail -2 gpurun_out/r5_path_parity.log
timeout -k 10 700 python3 -u tools/oracle_ray_scan.py cornell-lucy 1200 0 48 fp32 16 > gpurun_out/r5_ray_scan_c4.log 2>&1 || { tail -20 gpurun_out/r5_ray_scan_c4.log; exit 1; }
tail -2 gpurun_out/r5_ray_scan_c4.log
