#!/bin/bash
# prefetch re-record on a new model: GPU prefetch tests + BERT bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_prefetch_gpu.py > $O/g_pfchk_tests.txt 2>&1; rc=$?
tail -2 $O/g_pfchk_tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --model bert_base --seq 128 --steps 30 --warmup 5 --reference-config off --time-deterministic off > $O/g_pfchk_bert.json 2>/dev/null || exit 1
python -c "import json;print('bert', json.loads(open('$O/g_pfchk_bert.json').read().strip().splitlines()[-1])['value'])"
