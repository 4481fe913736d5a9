# Round measurement: parity tests, bench (default), rocprof kernel stats (--streams 1), PMC passes.
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench.err; exit $rc; }
timeout -k 10 300 python bench.py --mac-record --no-cpu-baseline > gpurun_out/bench_record.json 2>/dev/null
rc=$?; echo "bench record rc=$rc"; cat gpurun_out/bench_record.json; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R0/gpurun_out/prof/ktrace" -o run --output-format csv -- python "$R0/bench.py" --streams 1 --steps 200 --warmup 20 --no-cpu-baseline > "$R0/gpurun_out/prof/ktrace.json" 2> "$R0/gpurun_out/prof/ktrace.err"
rc=$?; echo "rocprof trace rc=$rc"; cat "$R0/gpurun_out/prof/ktrace.json"; python "$R0/tools/kstats.py" "$R0/gpurun_out/prof/ktrace/run_kernel_stats.csv"; [ $rc -ne 0 ] && exit $rc
rocprofv3 -L > "$R0/gpurun_out/prof/counters.txt" 2>&1 || true
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d "$R0/gpurun_out/prof/pmc_$C" -o run --output-format csv -- python "$R0/bench.py" --streams 1 --steps 50 --warmup 10 --no-cpu-baseline > "$R0/gpurun_out/prof/pmc_$C.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
cd "$R0" && python tools/pmc_to_json.py gpurun_out/prof/pmc_FETCH_SIZE gpurun_out/prof/pmc_WRITE_SIZE ${ROUND:-1} > gpurun_out/prof/pmc.json
rc=$?; cat gpurun_out/prof/pmc.json; exit $rc
