set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r5_final -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 10 --reference-config off --time-deterministic off > $O/prof_r5_final.txt 2>&1 || exit 1
echo done
