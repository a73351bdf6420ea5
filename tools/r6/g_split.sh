#!/bin/bash
# split-K conv plans: tests, fp32 reference-config plan table regenerated, A/B benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "split_k_plans or every_tile_config" tests/test_determinism_gpu.py > $O/g_split_tests.txt 2>&1; rc=$?
tail -3 $O/g_split_tests.txt
[ $rc -eq 0 ] || exit 1
REF="--model resnet18 --res 32 --classes 1000 --dtype fp32 --deterministic 1 --batch 1024 --reference-config off --time-deterministic off"
MIPIPE_SHIPPED_TUNE=0 timeout -k 10 300 python bench.py $REF --steps 3 --warmup 3 --tune 2 --save-tune $O/t_r18_f32.json > $O/g_split_gen.log 2>&1 || exit 1
echo table done
for r in 1 2; do
  MIPIPE_SHIPPED_TUNE=0 MIPIPE_TUNE_TABLE=$O/t_r18_f32.json timeout -k 10 200 python bench.py $REF --steps 20 --warmup 5 >> $O/g_split_ref.jsonl 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py $REF --steps 20 --warmup 5 >> $O/g_split_ref_old.jsonl 2>/dev/null || exit 1
done
python -c "import json;[print('new', json.loads(l)['value'], json.loads(l)['ms_per_step']) for l in open('$O/g_split_ref.jsonl') if l.startswith('{')];[print('old table', json.loads(l)['value'], json.loads(l)['ms_per_step']) for l in open('$O/g_split_ref_old.jsonl') if l.startswith('{')]"
timeout -k 10 300 python bench.py --reference-config off --time-deterministic off > $O/g_split_r50.jsonl 2>/dev/null || exit 1
python -c "import json;[print('r50', json.loads(l)['value'], json.loads(l)['ms_per_step']) for l in open('$O/g_split_r50.jsonl') if l.startswith('{')]"
echo done
