#!/bin/bash
# PMC passes (counters only with --kernel-trace) over one conv shape: tools/one_conv.py args.
# usage: bash tools/r4/pmc_conv.sh NAME N H Ci Co k s p op cfg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
name=$1; shift
O=$R/gpurun_out/pmc_$name
mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
pass() {
  local tag=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc "$@" \
     -d "$O/$tag" -o run -- python3 "$R/tools/one_conv.py" $ARGS > "$O/$tag.log" 2>&1)
}
ARGS="$*"
pass A SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU || exit 1
pass B SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE || exit 1
pass C FETCH_SIZE GRBM_COUNT || exit 1
python3 "$R/tools/pmc_summary.py" conv "$O/A" "$O/B" "$O/C" > "$O/summary.txt" 2>&1
cat "$O/summary.txt"
