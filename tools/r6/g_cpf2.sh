#!/bin/bash
# conv weights-only prefetch: tests, ResNet-50 default bench line A/B (MIPIPE_CONV_PREFETCH 1 vs 0), trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_determinism_gpu.py -k "conv or resnet or determin" > $O/g_cpf2_tests.txt 2>&1; rc=$?
tail -2 $O/g_cpf2_tests.txt
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for c in 1 0; do
    MIPIPE_CONV_PREFETCH=$c timeout -k 10 400 python bench.py > $O/g_cpf2_$c.$r.json 2>$O/g_cpf2_$c.$r.err || exit 1
    python -c "import json;d=json.loads(open('$O/g_cpf2_$c.$r.json').read().strip().splitlines()[-1]);print('conv_pf=$c', d['value'], d['deterministic_variant']['value'], d['reference_config']['value'])"
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p_cpf2_r50 -o run -- python bench.py --steps 5 --warmup 3 --reference-config off --time-deterministic off > $O/p_cpf2_r50.log 2>&1 || exit 1
echo done
