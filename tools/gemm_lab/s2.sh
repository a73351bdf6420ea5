cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python tools/tile_sweep.py --iters 8 > gpurun_out/tile_sweep_r4a.jsonl 2> gpurun_out/tile_sweep_r4a.err || exit 1
tail -1 gpurun_out/tile_sweep_r4a.jsonl
for d in 0 1 0 1; do
  timeout -k 10 300 python bench.py --model bert_base --steps 20 --warmup 5 --deterministic $d >> gpurun_out/b_bert_det.jsonl 2>/dev/null || exit 1
  tail -1 gpurun_out/b_bert_det.jsonl | cut -c1-150
done
