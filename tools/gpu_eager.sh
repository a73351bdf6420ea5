#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py --graph off > gpurun_out/eager.txt 2>gpurun_out/eager.err || exit $?
tail -1 gpurun_out/eager.txt
timeout -k 10 300 python bench.py --graph on > gpurun_out/graph.txt 2>gpurun_out/graph.err || exit $?
tail -1 gpurun_out/graph.txt
