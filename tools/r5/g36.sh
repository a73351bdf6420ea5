# BERT-base on the early-DMA build: bench x3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
rm -f $O/r5_bert_early.jsonl
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --model bert_base --seq 128 --steps 30 --warmup 10 --reference-config off --time-deterministic off >> $O/r5_bert_early.jsonl 2> $O/r5_bert_early.err || exit 1
done
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --reference-config off --time-deterministic off >> $O/r5_bert_early.jsonl 2>> $O/r5_bert_early.err || exit 1
echo done
