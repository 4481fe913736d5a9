# drop-in producer profile (per-phase us per batch)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_c
mkdir -p $O
timeout -k 10 300 python3 tools/dropin_bench.py --extra > $O/dropin.json 2> $O/dropin.err
echo "rc=$?" >> $O/done.txt
