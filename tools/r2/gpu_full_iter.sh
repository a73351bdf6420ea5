#!/bin/bash
# Full GPU suite (one process), then the 1-GPU bench + eager per-call kernel listing.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/full_iter_tests.txt 2>&1 || { tail -40 $O/full_iter_tests.txt; exit 1; }
tail -2 $O/full_iter_tests.txt
bash $R/tools/r2/gpu_percall.sh
