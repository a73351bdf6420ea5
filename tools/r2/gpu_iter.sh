#!/bin/bash
# Iteration check: selected GPU tests ($1 = pytest -k expression, "" = skip), then the 1-GPU
# ResNet-50 bench and an eager kernel-trace per-call listing (tools/r2/gpu_percall.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -n "$1" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > $O/iter_tests.txt 2>&1 || { tail -30 $O/iter_tests.txt; exit 1; }
  tail -2 $O/iter_tests.txt
fi
bash $R/tools/r2/gpu_percall.sh
