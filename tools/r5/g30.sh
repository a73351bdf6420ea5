# BERT-base with tile 14 available: bench x2 + kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
rm -f $O/r5_bert_now2.jsonl
for i in 1 2; do
timeout -k 10 300 python -u bench.py --model bert_base --seq 128 --steps 30 --warmup 10 --reference-config off --time-deterministic off 2>/dev/null >> $O/r5_bert_now2.jsonl || exit 1
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r5_bert2 -o run -- python $GRAFT_REPO_ROOT/bench.py --model bert_base --seq 128 --steps 5 --warmup 10 --reference-config off --time-deterministic off > $O/prof_r5_bert2.txt 2>&1 || exit 1
echo done
