# drop-in sweep: hugepage mempools (zero-copy), 4-KiB A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_f
mkdir -p $O
timeout -k 10 600 python3 tools/dropin_bench.py --extra > $O/dropin.json 2> $O/dropin.err
echo "rc=$?" >> $O/done.txt
