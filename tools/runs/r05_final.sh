# round 5, final tree: GPU suite, smoke, the driver's bench command (with PMC traffic, end-to-end and CPU
# baseline), a kernel trace of the bench (csv, for tools/kshapes.py) and a --multi-only trace, rocprofv3
# --stats of both
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_final
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
NBG_BENCH_FULL=$O/bench_full.json timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 bench.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace_multi -o run -- python3 bench.py --multi-only --steps 50 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline > $O/bench_multi.json 2> $O/bench_multi.err
echo "rc=$?" >> $O/done.txt
