# BERT-base after the tail-free / SGPR-pinned operand changes: bench x3 and the GEMM plan table
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
rm -f $O/r5_bert_now.jsonl
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --model bert_base --seq 128 --steps 30 --warmup 10 --reference-config off --time-deterministic off 2>/dev/null >> $O/r5_bert_now.jsonl || exit 1
done
timeout -k 10 600 python -u tools/gemm_plans.py > $O/r5_gemm_plans_bert2.jsonl 2> $O/r5_gemm_plans_bert2.err || exit 1
echo done
