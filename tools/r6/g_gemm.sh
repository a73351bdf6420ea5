#!/bin/bash
# fp32-output workspace split-K GEMM: tests, reference-config table regenerated, A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp32_gpu.py -k "gemm" > $O/g_gemm_tests.txt 2>&1; rc=$?
tail -3 $O/g_gemm_tests.txt
[ $rc -eq 0 ] || exit 1
REF="--model resnet18 --res 32 --classes 1000 --dtype fp32 --deterministic 1 --batch 1024 --reference-config off --time-deterministic off"
MIPIPE_SHIPPED_TUNE=0 timeout -k 10 300 python bench.py $REF --steps 3 --warmup 3 --tune 2 --save-tune $O/t_r18_f32_b.json > $O/g_gemm_gen.log 2>&1 || exit 1
for r in 1 2; do
  MIPIPE_SHIPPED_TUNE=0 MIPIPE_TUNE_TABLE=$O/t_r18_f32_b.json timeout -k 10 200 python bench.py $REF --steps 20 --warmup 5 >> $O/g_gemm_new.jsonl 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py $REF --steps 20 --warmup 5 >> $O/g_gemm_old.jsonl 2>/dev/null || exit 1
done
python -c "import json;[print('new', json.loads(l)['value']) for l in open('$O/g_gemm_new.jsonl') if l.startswith('{')];[print('old', json.loads(l)['value']) for l in open('$O/g_gemm_old.jsonl') if l.startswith('{')]"
echo done
