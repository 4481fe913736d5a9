# round 4 final tree: every GPU test, smoke(), the default bench line (as the driver runs it)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_f1
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 700 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "rc=$? seconds=$SECONDS" >> $O/done.txt
