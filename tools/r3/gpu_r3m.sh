#!/bin/bash
# one-shot IPC collectives (2 processes on one GPU) + native reducer at world 2 on GPU buckets
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3m
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 500 python3 -u -m pytest -v -x --timeout 240 --timeout-method thread tests/test_oneshot_gpu.py > $O/oneshot_tests.txt 2>&1 || { tail -60 $O/oneshot_tests.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/oneshot_tests.txt | tail -8
