# C3 (IMIX, 1000 backends, M=655373) variant timings + rocprof kernel stats
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python tools/kbench.py --mode 1 --nb 1000 --m 655373 --rounds 3 --iters 20 "$@" > gpurun_out/c3_kbench.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/c3_kbench.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R0/gpurun_out/c3prof" -o run --output-format csv -- python "$R0/tools/kbench.py" --mode 1 --nb 1000 --m 655373 --rounds 1 --iters 20 --no-multistream "$@" > "$R0/gpurun_out/c3prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; python "$R0/tools/kstats.py" "$R0/gpurun_out/c3prof/run_kernel_stats.csv"
exit $rc
