# round 6: 32-B staged windows for direct host batches (frame bytes 8..39), NBG_HOST_SLOTS 8, 64 server
# blocks: the GPU suite, then the drop-in sweep with its alternatives (48-B windows, depth 4, 32 blocks, ...)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_s
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 600 python3 tools/dropin_bench.py --extra > $O/dropin.json 2> $O/dropin.err
echo "rc=$?" >> $O/done.txt
