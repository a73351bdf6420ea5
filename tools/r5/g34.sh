# same box, same session: stock PyTorch-ROCm comparators next to mipipe (ResNet-50, BERT-base)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
rm -f $O/r5_same_box_stock.jsonl
timeout -k 10 500 python -u bench.py --impl stock --steps 20 --warmup 5 --reference-config off --time-deterministic off >> $O/r5_same_box_stock.jsonl 2> $O/r5_sbs_1.err || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --reference-config off --time-deterministic off >> $O/r5_same_box_stock.jsonl 2> $O/r5_sbs_2.err || exit 1
timeout -k 10 500 python -u bench.py --impl stock --model bert_base --seq 128 --steps 20 --warmup 5 --reference-config off --time-deterministic off >> $O/r5_same_box_stock.jsonl 2> $O/r5_sbs_3.err || exit 1
timeout -k 10 300 python -u bench.py --model bert_base --seq 128 --steps 20 --warmup 5 --reference-config off --time-deterministic off >> $O/r5_same_box_stock.jsonl 2> $O/r5_sbs_4.err || exit 1
echo done
