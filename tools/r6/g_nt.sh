#!/bin/bash
# ResNet-50 headline A/B of the non-temporal store size threshold (MIPIPE_NT_MIN_MB)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
B="--reference-config off --time-deterministic off --steps 30 --warmup 5"
for r in 1 2; do
  for t in 0 64 160; do
    MIPIPE_NT_MIN_MB=$t timeout -k 10 300 python bench.py $B > $O/g_nt_$t.$r.json 2>/dev/null || exit 1
    python -c "import json;print('$t', json.loads(open('$O/g_nt_$t.$r.json').read().strip().splitlines()[-1])['value'])"
  done
done
