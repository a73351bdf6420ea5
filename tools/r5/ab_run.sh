#!/bin/bash
# A/B on ONE box: runs `python bench.py ARGS` alternately with the in-tree _C and with the variant
# tools/r5/alt/NAME/_C*.so (a copy of the repo with that .so swapped in), ROUNDS times each.
# usage: bash tools/r5/ab_run.sh NAME ROUNDS OUT bench-args...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
name=$1; rounds=$2; out=$3; shift 3
ALT=/tmp/ab_$name
rm -rf $ALT && mkdir -p $ALT && cp -r $R/bench.py $R/kubeflow-v2-distributed-pytorch_amd $R/tools $ALT/ && ln -s kubeflow-v2-distributed-pytorch_amd $ALT/mipipe
cp $R/tools/r5/alt/$name/_C*.so $ALT/kubeflow-v2-distributed-pytorch_amd/
for i in $(seq $rounds); do
  (cd $R && timeout -k 10 300 python -u bench.py "$@" 2>/dev/null | sed "s/^/base /") >> $out || exit 1
  (cd $ALT && timeout -k 10 300 python -u bench.py "$@" 2>/dev/null | sed "s/^/$name /") >> $out || exit 1
done
