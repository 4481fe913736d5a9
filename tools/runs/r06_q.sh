# round 6: the host-batch server's block count at 16 pipelines now that the producers' gather is faster
# (threads dealt over the L3 caches), two rounds; 4 pipelines at 16 and 32 blocks
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_q
mkdir -p $O
timeout -k 10 500 python3 tools/dropin_bench.py --server-sweep > $O/sweep.json 2> $O/sweep.err
echo "rc=$?" >> $O/done.txt
