# Round measurement set: GPU parity, bench (C2 in place + records), rocprof kernel stats and PMC
# passes (tools/runs/gpu_bench.sh), then the C3/C5 config bench with its rocprof stats, and the
# end-to-end PCIe bench.  Everything lands in gpurun_out/.
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"
bash tools/runs/gpu_bench.sh || exit $?
echo "== configs"
timeout -k 10 400 python -u tools/config_bench.py > gpurun_out/configs.json 2> gpurun_out/configs.err
rc=$?; cat gpurun_out/configs.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/configs.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R0/gpurun_out/prof/cfg" -o run --output-format csv -- python "$R0/tools/config_bench.py" --streams 1 --steps 50 --warmup 5 > "$R0/gpurun_out/prof/cfg.json" 2> "$R0/gpurun_out/prof/cfg.err"
rc=$?; echo "rocprof configs rc=$rc"; python "$R0/tools/kstats.py" "$R0/gpurun_out/prof/cfg/run_kernel_stats.csv"; [ $rc -ne 0 ] && exit $rc
cd "$R0"
echo "== e2e"
timeout -k 10 300 python -u tools/e2e_bench.py > gpurun_out/e2e.json 2> gpurun_out/e2e.err
rc=$?; cat gpurun_out/e2e.json; exit $rc
