# 128x128 ping-pong tile (config 14): every-tile tests (bf16), single-op times, same-box bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "every_tile or every_plan or workspace_plans" > $O/r5_t14_tests.txt 2>&1 || exit 1
S="fwd:256,14,256,256,3,1,1:14 fwd:256,14,256,256,3,1,1:11 fwd:256,14,256,256,3,1,1:1 fwd:256,28,128,128,3,1,1:14 fwd:256,28,128,128,3,1,1:1 fwd:256,7,512,512,3,1,1:14 fwd:256,7,512,512,3,1,1:0 fwd:256,28,128,512,1,1,0:14 fwd:256,28,128,512,1,1,0:1 fwd:256,14,256,1024,1,1,0:14 fwd:256,14,256,1024,1,1,0:1 dgrad:256,14,256,256,3,1,1:14 dgrad:256,14,256,256,3,1,1:0 wgrad:256,14,256,1024,1,1,0:14 wgrad:256,14,256,1024,1,1,0:1"
rm -f $O/r5_t14_ops.jsonl
timeout -k 10 300 python -u tools/r5/conv_time.py t14 $S >> $O/r5_t14_ops.jsonl || exit 1
rm -f $O/r5_t14_ab.txt
bash tools/r5/env_ab.sh $O/r5_t14_ab.txt 3 MIPIPE_CONV_TILES=15 MIPIPE_CONV_TILES=14 -- --steps 30 --warmup 10 --reference-config off --time-deterministic off || exit 1
echo done
