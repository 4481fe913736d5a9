# round 6: batches in flight per pipeline (NBG_HOST_SLOTS now 8: depth 4 against 8) x server blocks (48, 64)
# at 16 pipelines, two rounds; one pipeline at depth 4 and 8
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_r
mkdir -p $O
timeout -k 10 500 python3 tools/dropin_bench.py --depth-sweep > $O/sweep.json 2> $O/sweep.err
echo "rc=$?" >> $O/done.txt
