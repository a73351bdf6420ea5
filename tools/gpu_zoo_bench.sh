#!/bin/bash
# Zoo throughput on one MI355X: mipipe (HIP kernels) vs stock PyTorch-ROCm on the same module tree.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/zoo_bench.jsonl
CFGS="${ZOO_CFGS:-mobilenet_v2 224 256;resnext50_32x4d 224 256;densenet121 224 256}"
IFS=';' read -ra LIST <<< "$CFGS"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  for impl in stock mipipe; do
    echo "start $1 $impl" >> gpurun_out/zoo_progress.txt
    timeout -k 10 500 python bench.py --model $1 --res $2 --batch $3 --steps 10 --warmup 3 --impl $impl > gpurun_out/zb.log 2>gpurun_out/zb.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "{\"model\": \"$1\", \"impl\": \"$impl\", \"rc\": $rc}" >> $out; tail -5 gpurun_out/zb.log gpurun_out/zb.err; exit $rc; fi
    tail -1 gpurun_out/zb.log >> $out
    echo "$1 $impl done"
  done
done
