# Round-2 measurement set: GPU parity + bench (PMC in run) + rocprof stats (tools/runs/gpu_bench.sh),
# the C++ small-batch bench (single-launch path, two-launch path), C3/C5 configs with their rocprof
# stats, and the end-to-end PCIe bench.  Everything lands in gpurun_out/.
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"
bash tools/runs/gpu_bench.sh || exit $?
echo "== small batches"
timeout -k 10 120 ./tools/small_bench > gpurun_out/small_new.json || exit $?
NBG_SMALL=0 timeout -k 10 120 ./tools/small_bench > gpurun_out/small_old.json || exit $?
cat gpurun_out/small_new.json gpurun_out/small_old.json
echo "== configs"
timeout -k 10 500 python -u tools/config_bench.py --cpu-baseline > gpurun_out/configs.json 2> gpurun_out/configs.err
rc=$?; cat gpurun_out/configs.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/configs.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R0/gpurun_out/prof/cfg" -o run --output-format csv -- python "$R0/tools/config_bench.py" --streams 1 --steps 50 --warmup 5 > "$R0/gpurun_out/prof/cfg.json" 2> "$R0/gpurun_out/prof/cfg.err"
rc=$?; echo "rocprof configs rc=$rc"; python "$R0/tools/kstats.py" "$R0/gpurun_out/prof/cfg/run_kernel_stats.csv"; [ $rc -ne 0 ] && exit $rc
cd "$R0"
echo "== e2e"
timeout -k 10 300 python -u tools/e2e_bench.py > gpurun_out/e2e.json 2> gpurun_out/e2e.err
rc=$?; cat gpurun_out/e2e.json; exit $rc
