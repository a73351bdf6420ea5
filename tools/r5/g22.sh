# where does a short-K 3x3 conv spend its time: base vs no-epilogue vs no-BN-stats builds
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
for v in noepi nostat; do
  ALT=/tmp/alt_$v
  rm -rf $ALT && mkdir -p $ALT && cp -r bench.py kubeflow-v2-distributed-pytorch_amd tools $ALT/ && ln -s kubeflow-v2-distributed-pytorch_amd $ALT/mipipe
  cp tools/r5/alt/$v/_C*.so $ALT/kubeflow-v2-distributed-pytorch_amd/
done
S="fwd:256,56,64,64,3,1,1:9 fwd:256,28,128,128,3,1,1:1 fwd:256,14,256,256,3,1,1:11 fwd:256,14,256,256,3,1,1:1 fwd:256,7,512,512,3,1,1:0 fwd:256,56,64,256,1,1,0:9 fwd:256,56,256,64,1,1,0:9 dgrad:256,56,64,64,3,1,1:9"
rm -f $O/r5_epi.jsonl
for i in 1 2; do
timeout -k 10 200 python -u tools/r5/conv_time.py base $S >> $O/r5_epi.jsonl || exit 1
for v in noepi nostat; do
(cd /tmp/alt_$v && timeout -k 10 200 python -u tools/r5/conv_time.py $v $S >> $O/r5_epi.jsonl) || exit 1
done
done
echo done
