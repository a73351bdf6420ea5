#!/bin/bash
# First GPU validation: kernel numerics, smoke, then (only if clean) bench + per-layer microbench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu > gpurun_out/gpu_tests.txt 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_tests.txt
tail -25 gpurun_out/gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1
rc=$?
echo "smoke rc=$rc" >> gpurun_out/smoke.txt
tail -3 gpurun_out/smoke.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python tools/bench_kernels.py --iters 5 > gpurun_out/bench_kernels.jsonl 2>gpurun_out/bench_kernels.err || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.txt 2>&1
echo "bench rc=$?" >> gpurun_out/bench.txt
tail -3 gpurun_out/bench.txt
