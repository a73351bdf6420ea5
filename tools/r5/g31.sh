# BERT: Linear weight-grads on a side stream (MIPIPE_SIDE_WGRAD_LINEAR) — same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
rm -f $O/r5_side_lin_ab.txt
bash tools/r5/env_ab.sh $O/r5_side_lin_ab.txt 3 MIPIPE_SIDE_WGRAD_LINEAR=1 MIPIPE_SIDE_WGRAD_LINEAR=0 -- --model bert_base --seq 128 --steps 30 --warmup 10 --reference-config off --time-deterministic off || exit 1
echo done
