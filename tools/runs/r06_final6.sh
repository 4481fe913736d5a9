# round 6, final tree (the replay and e2e mempools at a DPDK mbuf object stride): GPU suite, smoke, the driver's bench command (PMC traffic, end-to-end, drop-in,
# CPU baseline), kernel traces of the bench and of --multi-only (csv, for tools/kshapes.py), and the
# drop-in sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_final6
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
NBG_BENCH_FULL=$O/bench_full.json timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 bench.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace_multi -o run -- python3 bench.py --multi-only --steps 50 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline > $O/bench_multi.json 2> $O/bench_multi.err &&
timeout -k 10 600 python3 tools/dropin_bench.py --extra > $O/dropin.json 2> $O/dropin.err
echo "rc=$?" >> $O/done.txt
