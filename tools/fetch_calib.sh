#!/bin/bash
# FETCH_SIZE calibration (tools/fetch_calib/fetch_calib.hip): the counter
# passes of the microkernel patterns, then the same request counters of the
# production kernels on the bench workload (one step, one stream).  Each pass
# its own rocprofv3 run with its own time limit.  Output: gpurun_out/calib/;
# tools/fetch_calib.py turns it into profiles/r06_fetch_calib.txt.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/calib}
mkdir -p $OUT
bin=tools/fetch_calib/fetch_calib
$bin 65536 1 > $OUT/order.json || exit 1
pass() {   # name, then counters
  name=$1; shift
  timeout -s KILL 60 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o p -- $bin 65536 3 > $OUT/$name.out 2> $OUT/$name.err
  echo "pass $name rc=$?"
}
pass fetch FETCH_SIZE
pass req TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_MISS_sum TCC_HIT_sum
pass bubble TCC_BUBBLE_sum
pass write WRITE_SIZE
# the production kernels: the same request counters (bench.py's PMC child)
for grp in "req TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_MISS_sum TCC_HIT_sum" "bubble TCC_BUBBLE_sum" "fetch FETCH_SIZE"; do
  set -- $grp; name=bench_$1; shift
  RTGPU_STREAMS=1 timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o p -- \
    python3 bench.py --pmc-child > $OUT/$name.out 2> $OUT/$name.err
  echo "pass $name rc=$?"
done
python3 tools/fetch_calib.py $OUT
