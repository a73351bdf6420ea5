#!/bin/bash
# regenerate the ResNet-50 deterministic plan table on this tree (split-K plans now candidates),
# A/B the deterministic variant, profile the reference config after split-K
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
MIPIPE_SHIPPED_TUNE=0 timeout -k 10 400 python bench.py --deterministic 1 --tune 2 --steps 3 --warmup 3 --reference-config off --time-deterministic off --save-tune $O/t_r50_det.json > $O/g_tab_gen.log 2>&1 || exit 1
echo table done
for r in 1 2; do
  MIPIPE_SHIPPED_TUNE=0 MIPIPE_TUNE_TABLE=$O/t_r50_det.json timeout -k 10 200 python bench.py --deterministic 1 --reference-config off --time-deterministic off >> $O/g_tab_new.jsonl 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --deterministic 1 --reference-config off --time-deterministic off >> $O/g_tab_old.jsonl 2>/dev/null || exit 1
done
python -c "import json;[print('new', json.loads(l)['value']) for l in open('$O/g_tab_new.jsonl') if l.startswith('{')];[print('old', json.loads(l)['value']) for l in open('$O/g_tab_old.jsonl') if l.startswith('{')]"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_ref3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet18 --res 32 --classes 1000 --dtype fp32 --deterministic 1 --batch 1024 --steps 5 --warmup 5 --reference-config off --time-deterministic off > $O/p_ref3.log 2>&1 || exit 1
echo done
