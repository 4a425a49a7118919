#!/bin/bash
# Round 3: C4 with the lean k_shade at 7 waves (lib): 2 vs 3 twin streams,
# without the prefetched next ray (lib_nopf: lanes claim only when idle), and
# with twin 1 starting after twin 0's first k_extend (RTGPU_TWIN_OFFSET).
set -o pipefail
OUT=gpurun_out/r3i
mkdir -p $OUT
b() {   # name lib streams
  RTGPU_STREAMS=$3 RTGPU_LIB_DIR=$2 timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs \
    --no-three-pass --no-pmc --no-balance > $OUT/$1.json 2> $OUT/$1.err || { echo "bench $1 failed"; tail -20 $OUT/$1.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'], {k: v['ms_avg'] for k, v in d['kernels'].items()})" $OUT/$1.json $1
}
timeout -k 10 200 python3 tools/multidev_diag.py 25 > $OUT/multidev_diag.log 2>&1 || { tail -20 $OUT/multidev_diag.log; exit 1; }
tail -1 $OUT/multidev_diag.log
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for rep in 1 2; do
  b s2.$rep lib 2 || exit 1
  b s3.$rep lib 3 || exit 1
  b nopf.$rep lib_nopf 2 || exit 1
  RTGPU_TWIN_OFFSET=1 b off.$rep lib 2 || exit 1
done
echo r3i-done
