#!/bin/bash
# Same-box comparison: mipipe bench.py vs stock PyTorch-ROCm (bench.py --impl stock: MIOpen,
# channels_last, bf16 autocast / fp32, torch SGD) for ResNet-50 b256 bf16 and ResNet-18 CIFAR fp32.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1; shift; timeout -k 10 400 python3 $R/bench.py "$@" > $O/sb_$name.txt 2>&1 || { tail -20 $O/sb_$name.txt; exit 1; }; echo "$name $(tail -1 $O/sb_$name.txt | cut -c1-160)"; }
run r50_mipipe --steps 20 --warmup 5
run r50_stock --impl stock --steps 20 --warmup 5
run r18fp32_mipipe --model resnet18 --res 32 --batch 1024 --classes 10 --dtype fp32 --steps 30 --warmup 5
run r18fp32_stock --impl stock --model resnet18 --res 32 --batch 1024 --classes 10 --dtype fp32 --steps 30 --warmup 5
