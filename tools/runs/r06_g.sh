# coalesced small-kernel loads + MAC swap in the host gather: the GPU suite, then the drop-in sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_g
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 600 python3 tools/dropin_bench.py --extra > $O/dropin.json 2> $O/dropin.err
echo "rc=$?" >> $O/done.txt
