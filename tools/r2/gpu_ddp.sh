#!/bin/bash
# RCCL DDP on one GPU (force_reduce), graph capture under DDP, kernel trace for overlap.
set -o pipefail
mkdir -p gpurun_out/r2
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r2/ddp_tests.txt 2>&1 || { tail -40 gpurun_out/r2/ddp_tests.txt; exit 1; }
tail -5 gpurun_out/r2/ddp_tests.txt
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29511 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0
for g in off on; do
  timeout -k 10 200 python bench.py --force-reduce --graph $g --steps 20 --warmup 5 > gpurun_out/r2/bench_fr_$g.txt 2>&1 || exit $?
  tail -1 gpurun_out/r2/bench_fr_$g.txt
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r2/prof_ddp -o run -- python3 $R/bench.py --force-reduce --graph off --steps 3 --warmup 2 > $R/gpurun_out/r2/prof_ddp.txt 2>&1 || exit $?
echo prof-ok
