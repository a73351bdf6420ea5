cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > gpurun_out/t_gemm.log 2>&1 || { tail -30 gpurun_out/t_gemm.log; exit 1; }
tail -2 gpurun_out/t_gemm.log
timeout -k 10 600 python tools/gemm_plans.py > gpurun_out/gemm_plans_r4b.jsonl 2> gpurun_out/gemm_plans_r4b.err || { tail gpurun_out/gemm_plans_r4b.err; exit 1; }
cut -c1-120 gpurun_out/gemm_plans_r4b.jsonl
for i in 1 2; do
timeout -k 10 300 python bench.py --model bert_base --steps 20 --warmup 5 --save-tune gpurun_out/tune_bert_nolib.json >> gpurun_out/b_bert_nolib.jsonl 2>/dev/null || exit 1
tail -1 gpurun_out/b_bert_nolib.jsonl | cut -c1-120
done
