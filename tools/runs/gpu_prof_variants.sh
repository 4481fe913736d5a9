# rocprofv3 kernel stats of bench.py's single-stream pass with the records and read-only variants
# (each variant is its own classify_stream_kernel<F4, HIST, MODE> instantiation: MODE 1 in place,
# 2 records, 0 read-only).
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R0/gpurun_out/prof/var" -o run --output-format csv -- python "$R0/bench.py" --inline --no-pmc --no-cpu-baseline --streams 1 --steps 200 --warmup 20 > "$R0/gpurun_out/prof/var.json" 2> "$R0/gpurun_out/prof/var.err"
rc=$?; echo "rocprof rc=$rc"; cat "$R0/gpurun_out/prof/var.json"; python "$R0/tools/kstats.py" "$R0/gpurun_out/prof/var/run_kernel_stats.csv"; exit $rc
