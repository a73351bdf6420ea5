#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/ -q -m gpu > gpurun_out/gpu_tests.txt 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_tests.txt
tail -12 gpurun_out/gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.txt 2>&1 || exit $?
tail -1 gpurun_out/bench.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.txt 2>&1
echo "prof rc=$?"
