#!/bin/bash
# LDS-level folded BN: bit-exactness tests, same-box end-to-end A/B of the size-gated "auto" mode
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bn_fold_gpu.py > $O/g_fold3_tests.txt 2>&1; rc=$?
tail -3 $O/g_fold3_tests.txt
[ $rc -eq 0 ] || exit 1

for r in 1 2 3; do
  MIPIPE_BN_FOLD=0 timeout -k 10 200 python bench.py --reference-config off --time-deterministic off --steps 30 --warmup 10 >> $O/g_fold3_ab.txt 2>/dev/null && echo "A(off)" &&
  MIPIPE_BN_FOLD=auto timeout -k 10 200 python bench.py --reference-config off --time-deterministic off --steps 30 --warmup 10 >> $O/g_fold3_ab.txt 2>/dev/null && echo "B(fold)" || exit 1
done
python -c "import json;[print(json.loads(l)['value'], json.loads(l)['ms_per_step']) for l in open('$O/g_fold3_ab.txt') if l.startswith('{')]"
echo done
