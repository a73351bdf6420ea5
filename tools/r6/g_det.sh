#!/bin/bash
# deterministic-reduction launches folded: tests + reference-config bench + its kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_determinism_gpu.py tests/test_fp32_gpu.py tests/test_stem_fused_gpu.py tests/test_kernels_gpu.py -k "det or fp32 or pool_bn or stem or finalize or bn" > $O/g_det_tests.txt 2>&1; rc=$?
tail -3 $O/g_det_tests.txt
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
timeout -k 10 200 python bench.py --model resnet18 --res 32 --classes 1000 --dtype fp32 --deterministic 1 --batch 1024 --steps 20 --warmup 5 --reference-config off --time-deterministic off >> $O/g_det_ref.jsonl 2>/dev/null || exit 1
done
python -c "import json;[print(json.loads(l)['value'], json.loads(l)['ms_per_step']) for l in open('$O/g_det_ref.jsonl') if l.startswith('{')]"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_ref2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet18 --res 32 --classes 1000 --dtype fp32 --deterministic 1 --batch 1024 --steps 5 --warmup 5 --reference-config off --time-deterministic off > $O/p_ref2.log 2>&1 || exit 1
echo done
