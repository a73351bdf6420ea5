#!/bin/bash
# Conv operand prefetch: tests, ResNet-50 default bench line A/B (MIPIPE_PREFETCH 1 vs 0), trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_prefetch_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_determinism_gpu.py tests/test_fp32_gpu.py -k "prefetch or conv or resnet or determin or gemm" > $O/g_cpf_tests.txt 2>&1; rc=$?
tail -3 $O/g_cpf_tests.txt
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
  timeout -k 10 400 python bench.py > $O/g_cpf_on_$r.json 2>$O/g_cpf_on_$r.err || exit 1
  tail -1 $O/g_cpf_on_$r.json | cut -c1-200
  MIPIPE_PREFETCH=0 timeout -k 10 400 python bench.py > $O/g_cpf_off_$r.json 2>$O/g_cpf_off_$r.err || exit 1
  tail -1 $O/g_cpf_off_$r.json | cut -c1-200
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p_cpf_r50 -o run -- python bench.py --steps 5 --warmup 3 --reference-config off --time-deterministic off > $O/p_cpf_r50.log 2>&1 || exit 1
echo done
