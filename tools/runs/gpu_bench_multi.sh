# The default bench (with the multi-batch variants) and rocprof kernel stats of the multi-batch
# launches alone and of the single-batch variants pass.
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 500 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R0/gpurun_out/prof/multi" -o run --output-format csv -- python "$R0/bench.py" --inline --no-pmc --no-cpu-baseline --multi-only --steps 200 > "$R0/gpurun_out/prof/multi.json" 2> "$R0/gpurun_out/prof/multi.err"
rc=$?; echo "rocprof multi rc=$rc"; cat "$R0/gpurun_out/prof/multi.json"; python "$R0/tools/kstats.py" "$R0/gpurun_out/prof/multi/run_kernel_stats.csv"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R0/gpurun_out/prof/var" -o run --output-format csv -- python "$R0/bench.py" --inline --no-pmc --no-cpu-baseline --no-multi --streams 1 --steps 200 --warmup 20 > "$R0/gpurun_out/prof/var.json" 2> "$R0/gpurun_out/prof/var.err"
rc=$?; echo "rocprof variants rc=$rc"; python "$R0/tools/kstats.py" "$R0/gpurun_out/prof/var/run_kernel_stats.csv"; exit $rc
