# round 6: drop-in thread placement A/B at 16 pipelines (dealt over the L3 caches of the GPU's socket, or
# packed on the first cores), 3 alternating rounds, plus 4 pipelines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_p
mkdir -p $O
timeout -k 10 500 python3 tools/dropin_bench.py --ab-spread > $O/ab.json 2> $O/ab.err
echo "rc=$?" >> $O/done.txt
