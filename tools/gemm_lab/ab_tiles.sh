cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for t in 14 11 14; do
  MIPIPE_CONV_TILES=$t timeout -k 10 300 python bench.py --steps 20 --warmup 5 --save-tune gpurun_out/tune_r50_$t.json >> gpurun_out/b_r50.jsonl 2>gpurun_out/b_r50_$t.err || exit 1
  tail -1 gpurun_out/b_r50.jsonl | cut -c1-160
done
for t in 14 11; do
  MIPIPE_CONV_TILES=$t timeout -k 10 300 python bench.py --model bert_base --steps 20 --warmup 5 --save-tune gpurun_out/tune_bert_$t.json >> gpurun_out/b_bert.jsonl 2>gpurun_out/b_bert_$t.err || exit 1
  tail -1 gpurun_out/b_bert.jsonl | cut -c1-160
done
