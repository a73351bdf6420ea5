#!/bin/bash
# Per-kernel HBM bytes (TCC FETCH_SIZE / WRITE_SIZE, one counter group per run) for a ResNet-50
# b256 training step (eager), joined with the kernel durations of the same runs.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2/bytes
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --steps 2 --warmup 3 --graph off --tune 1 > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py --steps 2 --warmup 3 --graph off --tune 1 > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
ls $O/fetch $O/write
