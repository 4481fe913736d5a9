# round 6: the drop-in path by mempool size (one 10k-frame capture against 64k mbufs per pipeline) with and
# without the per-task / per-phase timers (now TSC reads), at 1, 4 and 16 pipelines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_m
mkdir -p $O
timeout -k 10 500 python3 tools/dropin_bench.py --pool-sweep > $O/pool.json 2> $O/pool.err
echo "rc=$?" >> $O/done.txt
