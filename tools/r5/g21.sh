# does LDS-DMA traffic of the im2col A operand bound the 3x3 convs?  base vs a build whose A
# descriptor has zero records (every A load returns zeros without memory traffic)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
ALT=/tmp/alt_noa
rm -rf $ALT && mkdir -p $ALT && cp -r bench.py kubeflow-v2-distributed-pytorch_amd tools $ALT/ && ln -s kubeflow-v2-distributed-pytorch_amd $ALT/mipipe
cp tools/r5/alt/noa/_C*.so $ALT/kubeflow-v2-distributed-pytorch_amd/
S="fwd:256,56,64,64,3,1,1:9 fwd:256,56,64,64,3,1,1:2 fwd:256,28,128,128,3,1,1:1 fwd:256,28,128,128,3,1,1:9 fwd:256,14,256,256,3,1,1:11 fwd:256,14,256,256,3,1,1:1 fwd:256,7,512,512,3,1,1:0 fwd:256,7,512,512,3,1,1:1 dgrad:256,56,64,64,3,1,1:9 dgrad:256,14,256,256,3,1,1:0"
rm -f $O/r5_noa.jsonl
for i in 1 2; do
timeout -k 10 200 python -u tools/r5/conv_time.py base $S >> $O/r5_noa.jsonl || exit 1
(cd $ALT && timeout -k 10 200 python -u tools/r5/conv_time.py noa $S >> $O/r5_noa.jsonl) || exit 1
done
echo done
