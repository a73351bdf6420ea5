#!/bin/bash
# DDP rehearsal on one GPU (2 gloo ranks) for ResNet-18 and zoo architectures
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in "resnet18 32" "mobilenet_v2 64" "resnext50_32x4d 64" "googlenet 64" "shufflenet_v2_x1_0 64"; do
  set -- $cfg
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29533 tools/ddp_gpu_check.py --arch $1 --res $2 >> gpurun_out/ddp_zoo.txt 2>&1 || { tail -20 gpurun_out/ddp_zoo.txt; exit 1; }
  grep -E "OK|info" gpurun_out/ddp_zoo.txt | tail -3
done
