# group kernel duration per scan mode (rocprof, single stream full path), then the multi-stream A/B
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for G in ${GSCAN:-2 1}; do
  NBG_GSCAN=$G timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R0/gpurun_out/gp$G" -o run --output-format csv -- python "$R0/tools/kbench.py" --no-multistream --rounds 2 --only "full path inplace,classify inplace nogroup" "$@" > "$R0/gpurun_out/gp$G.log" 2>&1
  rc=$?; echo "== GSCAN=$G (rc=$rc)"; grep median "$R0/gpurun_out/gp$G.log"; python "$R0/tools/kstats.py" "$R0/gpurun_out/gp$G/run_kernel_stats.csv" | grep -v rocclr
  [ $rc -ne 0 ] && exit $rc
done
cd "$R0"
for G in ${GSCAN:-2 1}; do
  NBG_GSCAN=$G timeout -k 10 300 python tools/kbench.py --only "x2 streams,x4 streams" "$@" > gpurun_out/kb$G.log 2>&1
  rc=$?; echo "== GSCAN=$G multistream"; grep median gpurun_out/kb$G.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
