# Round-2 bench check: CPU inventory of the box, the default bench (launcher, PMC passes,
# variants, CPU baseline), and the rocprof kernel stats of the same workload (single stream).
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
echo "nproc $(nproc) affinity $(python -c 'import os; print(len(os.sched_getaffinity(0)))') cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
timeout -k 10 500 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R0/gpurun_out/prof/ktrace" -o run --output-format csv -- python "$R0/bench.py" --inline --no-pmc --no-cpu-baseline --no-variants --streams 1 --steps 200 --warmup 20 > "$R0/gpurun_out/prof/ktrace.json" 2> "$R0/gpurun_out/prof/ktrace.err"
rc=$?; echo "rocprof trace rc=$rc"; cat "$R0/gpurun_out/prof/ktrace.json"; python "$R0/tools/kstats.py" "$R0/gpurun_out/prof/ktrace/run_kernel_stats.csv"; exit $rc
