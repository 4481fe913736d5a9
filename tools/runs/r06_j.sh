# full GPU suite (host-batch server, 4 slots), smoke, the drop-in sweep with extras, then the driver's bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_j
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 600 python3 tools/dropin_bench.py --extra > $O/dropin.json 2> $O/dropin.err &&
NBG_BENCH_FULL=$O/bench_full.json timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "rc=$?" >> $O/done.txt
