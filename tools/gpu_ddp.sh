#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/ddp_gpu_check.py > gpurun_out/ddp_check.txt 2>&1
rc=$?
tail -5 gpurun_out/ddp_check.txt
exit $rc
