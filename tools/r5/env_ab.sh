#!/bin/bash
# Same-box A/B of environment settings: ROUNDS x (each setting in turn) of python bench.py ARGS.
# usage: bash tools/r5/env_ab.sh OUT ROUNDS "VAR=a" "VAR=b" ... -- bench-args...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
out=$1; rounds=$2; shift 2
sets=()
while [ "$1" != "--" ]; do sets+=("$1"); shift; done
shift
for i in $(seq $rounds); do
  for st in "${sets[@]}"; do
    tag=$(echo "$st" | tr '/ ' '_+')
    (cd $R && env $st timeout -k 10 300 python -u bench.py "$@" 2>/dev/null | sed "s|^|$tag |") >> $out || exit 1
  done
done
