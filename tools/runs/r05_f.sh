# round 5 (session 2): re-check of the restored tree: GPU suite, smoke, the driver's bench command,
# then a kernel trace of the bench (no PMC) for per-kernel times
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_f
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err
echo "rc=$?" >> $O/done.txt
timeout -k 10 180 python3 tools/gprobe.py run > $O/gprobe.txt 2>&1
echo "rc_gprobe=$?" >> $O/done.txt
timeout -k 10 60 ./tools/groupfloor 200 > $O/groupfloor.txt 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/floorprof -o run -- ./tools/groupfloor 200 > $O/groupfloor_prof.txt 2>&1
echo "rc_floor=$?" >> $O/done.txt
