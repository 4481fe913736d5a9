# round 6: the drop-in path by mempool size (mbufs per pipeline's LoopPort: one 10k-frame capture, two,
# and the 64k default so far) at 1, 4 and 16 pipelines through the host-batch server
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_l
mkdir -p $O
timeout -k 10 500 python3 tools/dropin_bench.py --pool-sweep > $O/pool.json 2> $O/pool.err
echo "rc=$?" >> $O/done.txt
