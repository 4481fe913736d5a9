# Round measurement: parity tests, the default bench (launcher, in-run PMC traffic, variants, CPU
# baseline), and the rocprof kernel stats of the same workload on one stream.
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R0/gpurun_out/prof/ktrace" -o run --output-format csv -- python "$R0/bench.py" --inline --no-pmc --no-cpu-baseline --no-variants --streams 1 --steps 200 --warmup 20 > "$R0/gpurun_out/prof/ktrace.json" 2> "$R0/gpurun_out/prof/ktrace.err"
rc=$?; echo "rocprof trace rc=$rc"; cat "$R0/gpurun_out/prof/ktrace.json"; python "$R0/tools/kstats.py" "$R0/gpurun_out/prof/ktrace/run_kernel_stats.csv"; exit $rc
