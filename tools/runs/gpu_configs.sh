# C3 / C5 config throughput + rocprof kernel stats (single stream)
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python tools/config_bench.py "$@" > gpurun_out/configs.json 2> gpurun_out/configs.err
rc=$?; cat gpurun_out/configs.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/configs.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$R0/gpurun_out/cfgprof" -o run --output-format csv -- python "$R0/tools/config_bench.py" --streams 1 --steps 50 --warmup 5 > "$R0/gpurun_out/cfgprof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; python "$R0/tools/kstats.py" "$R0/gpurun_out/cfgprof/run_kernel_stats.csv"
exit $rc
