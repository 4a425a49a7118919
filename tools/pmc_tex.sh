#!/bin/bash
# Vector-memory pipeline counters (TA address unit, TD data unit, TCP vector
# L1 and its address translation) of bench.py's default workload, one pass
# per counter group, for each node format given (default: fp32 quant8;
# NODES="fp32 wide8" for the 8-wide comparison).
# Output: gpurun_out/pmc_tex/<nodes>/<pass>/; summarise with
#   python3 tools/pmc_summary.py gpurun_out/pmc_tex/<nodes>
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_tex}
ARGS=${ARGS:---steps 1 --warmup 0 --no-cpu-baseline --no-count --no-configs --no-balance --no-three-pass --no-pmc}
for nodes in ${NODES:-fp32 quant8}; do
  mkdir -p $OUT/$nodes
  run() {
    name=$1; shift
    RTGPU_STREAMS=1 timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$nodes/$name -o p -- \
      python3 bench.py $ARGS --nodes $nodes > $OUT/$nodes/$name.json 2> $OUT/$nodes/$name.err
  }
  run ta TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
  run td TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE
  run tcp1 TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
  run tcp2 TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum
  run sq SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
  run valu SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
done
