#!/bin/bash
# two-stage fp32 main loop: fp32 numerics tests, reference-config bench, kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fp32_gpu.py tests/test_determinism_gpu.py tests/test_kernels_gpu.py -k "fp32 or f32 or det or every or split" > $O/g_f32_tests.txt 2>&1; rc=$?
tail -3 $O/g_f32_tests.txt
[ $rc -eq 0 ] || exit 1
REF="--model resnet18 --res 32 --classes 1000 --dtype fp32 --deterministic 1 --batch 1024 --reference-config off --time-deterministic off"
for r in 1 2; do
  timeout -k 10 200 python bench.py $REF --steps 20 --warmup 5 >> $O/g_f32_ref.jsonl 2>/dev/null || exit 1
done
python -c "import json;[print(json.loads(l)['value'], json.loads(l)['ms_per_step']) for l in open('$O/g_f32_ref.jsonl') if l.startswith('{')]"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_ref5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py $REF --steps 5 --warmup 5 > $O/p_ref5.log 2>&1 || exit 1
echo done
