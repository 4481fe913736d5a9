# round 6, first call: the whole GPU suite (new: bench-shape C3/C5 parity with owned windows, ring grouping at
# 200 backends, ring stop twice), smoke, and the driver's bench command (imix_output_checks)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_a
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
NBG_BENCH_FULL=$O/bench_full.json timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "rc=$?" >> $O/done.txt
