#!/bin/bash
# End-of-round evidence: ResNet-50 kernel stats (no graph replay, per-kernel accounting),
# ResNet-18 CIFAR reference-config bench line, ResNet-50 graphed bench line.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r50.txt 2>&1 || exit $?
tail -1 gpurun_out/bench_r50.txt
timeout -k 10 200 python bench.py --model resnet18 --res 32 --batch 1024 --steps 30 --warmup 5 > gpurun_out/bench_r18.txt 2>&1 || exit $?
tail -1 gpurun_out/bench_r18.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --graph off > $R/gpurun_out/prof_bench.txt 2>&1 || exit $?
echo "prof ok"
