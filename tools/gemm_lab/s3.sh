cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python tools/gemm_plans.py > gpurun_out/gemm_plans_r4.jsonl 2> gpurun_out/gemm_plans_r4.err || { tail gpurun_out/gemm_plans_r4.err; exit 1; }
cut -c1-150 gpurun_out/gemm_plans_r4.jsonl
timeout -k 10 300 python bench.py --model bert_base --steps 10 --warmup 3 --deterministic 1 --tune 2 --save-tune gpurun_out/tune_bert_det.json > /dev/null 2>&1 || exit 1
for d in 1 0 1; do
  MIPIPE_TUNE_TABLE=gpurun_out/tune_bert_det.json timeout -k 10 300 python bench.py --model bert_base --steps 20 --warmup 5 --deterministic $d >> gpurun_out/b_bert_det2.jsonl 2>/dev/null || exit 1
  tail -1 gpurun_out/b_bert_det2.jsonl | cut -c1-150
done
