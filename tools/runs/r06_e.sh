# drop-in sweep with a hardware queue per pipeline, coarse-grained staging A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_e
mkdir -p $O
timeout -k 10 600 python3 tools/dropin_bench.py --extra > $O/dropin.json 2> $O/dropin.err
echo "rc=$?" >> $O/done.txt
