set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_trace_deep
mkdir -p $O
# kernel trace of individual conv ops (20 calls each)
for spec in "256 14 256 1024 1 1 0 wgrad" "256 14 1024 256 1 1 0 wgrad" "256 56 64 256 1 1 0 wgrad" "256 14 256 1024 1 1 0 fwd" "256 56 256 64 1 1 0 fwd" "256 14 256 256 3 1 1 fwd"; do
  tag=$(echo $spec | tr ' ' '_')
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 $GRAFT_REPO_ROOT/tools/one_conv.py $spec > $O/$tag.log 2>&1) || exit 1
done
bash tools/r4/pmc_conv.sh r5_l3c3_wgrad 256 14 256 1024 1 1 0 wgrad -1 > /dev/null 2>&1 || exit 1
bash tools/r4/pmc_conv.sh r5_l1c3_wgrad 256 56 64 256 1 1 0 wgrad -1 > /dev/null 2>&1 || exit 1
bash tools/r4/pmc_conv.sh r5_l3c3_fwd 256 14 256 1024 1 1 0 fwd -1 > /dev/null 2>&1 || exit 1
echo done
