#!/bin/bash
# Texture-address / L1 pressure of one conv shape: is the LDS-DMA operand path the limiter?
# usage: bash tools/r5/pmc_ta.sh NAME N H Ci Co k s p op cfg   (tools/one_conv.py args)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
name=$1; shift
O=$R/gpurun_out/pmcta_$name
mkdir -p "$O"
ARGS="$*"
pass() {
  local tag=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc "$@" \
     -d "$O/$tag" -o run -- python3 "$R/tools/one_conv.py" $ARGS > "$O/$tag.log" 2>&1)
}
pass A TA_BUSY_avr TA_BUFFER_READ_LDS_WAVEFRONTS_sum GRBM_GUI_ACTIVE || exit 1
pass B TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE || exit 1
pass C TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE || exit 1
pass D SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE || exit 1
python3 "$R/tools/pmc_summary.py" conv "$O/A" "$O/B" "$O/C" "$O/D" > "$O/summary.txt" 2>&1
cat "$O/summary.txt"
