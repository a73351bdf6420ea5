#!/bin/bash
# tests + ResNet-50 and BERT benches (one GPU call)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/ -q -m gpu > gpurun_out/gpu_tests.txt 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_tests.txt
tail -5 gpurun_out/gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.txt 2>&1 || exit $?
tail -1 gpurun_out/bench.txt
timeout -k 10 300 python bench.py --model bert_base --steps 10 --warmup 3 > gpurun_out/bench_bert.txt 2>&1 || exit $?
tail -1 gpurun_out/bench_bert.txt
