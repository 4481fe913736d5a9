# drop-in tuning: host-gather prefetch distance, server blocks, depth
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_i
mkdir -p $O
timeout -k 10 600 python3 tools/dropin_bench.py --tune > $O/dropin.json 2> $O/dropin.err
echo "rc=$?" >> $O/done.txt
