# counter list (TA / TD / TCP / SQ LDS) for the LDS-DMA throughput question
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 -L > $O/r5_counters_list.txt 2>&1 || exit 1
echo done
