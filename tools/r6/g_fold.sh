#!/bin/bash
# folded BN2 -> conv3: bit-exactness tests, model tests, same-box A/B, kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bn_fold_gpu.py tests/test_model_gpu.py tests/test_determinism_gpu.py > $O/g_fold_tests.txt 2>&1; rc=$?
tail -3 $O/g_fold_tests.txt
[ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  MIPIPE_BN_FOLD=0 timeout -k 10 200 python bench.py --reference-config off --time-deterministic off --steps 30 --warmup 10 >> $O/g_fold_ab.txt 2>/dev/null && echo "A(off)" &&
  MIPIPE_BN_FOLD=1 timeout -k 10 200 python bench.py --reference-config off --time-deterministic off --steps 30 --warmup 10 >> $O/g_fold_ab.txt 2>/dev/null && echo "B(fold)" || exit 1
done
python -c "import json;[print(json.loads(l)['value'], json.loads(l)['ms_per_step']) for l in open('$O/g_fold_ab.txt') if l.startswith('{')]"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_fold -o run -- python3 $GRAFT_REPO_ROOT/bench.py --reference-config off --time-deterministic off --steps 3 --warmup 5 > $O/p_fold.log 2>&1 || exit 1
echo done
