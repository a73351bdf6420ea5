#!/bin/bash
# Stock PyTorch-ROCm comparator sweep on 1 MI355X (each step time-limited).
set -o pipefail
mkdir -p gpurun_out
ls -la mipipe > gpurun_out/symlink_check.txt 2>&1
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
O=gpurun_out/stock.jsonl
: > $O
timeout -k 10 300 python tools/stock_baseline.py --model resnet50 --batch 256 --dtype bf16 --steps 20 --warmup 5 >> $O 2>gpurun_out/stock_err1.txt && \
timeout -k 10 200 python tools/stock_baseline.py --model resnet18 --batch 1024 --res 32 --dtype fp32 --steps 20 --warmup 5 >> $O 2>gpurun_out/stock_err2.txt && \
timeout -k 10 200 python tools/stock_baseline.py --model resnet18 --batch 1024 --res 32 --dtype bf16 --steps 20 --warmup 5 >> $O 2>gpurun_out/stock_err3.txt && \
timeout -k 10 300 python tools/stock_baseline.py --model resnet50 --batch 256 --dtype fp32 --steps 10 --warmup 3 >> $O 2>gpurun_out/stock_err4.txt
cat $O
