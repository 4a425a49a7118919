#!/bin/bash
# PMC passes (one counter group per pass, never combined with tracing) of
# bench.py on the default workload (one step).  Output: gpurun_out/pmc/<pass>/
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
ARGS=${ARGS:---steps 1 --warmup 0 --no-cpu-baseline --no-count --no-configs --no-balance --no-three-pass}
mkdir -p $OUT
run() {
  name=$1; shift
  RTGPU_STREAMS=1 timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o p -- python3 bench.py $ARGS > $OUT/$name.json 2> $OUT/$name.err
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sq2 SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD
run tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
run tcp TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum


