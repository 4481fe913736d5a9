# rocprof kernel trace of selected kbench variants (single stream), per-kernel stats
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp
i=0
for V in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R0/gpurun_out/kp$i" -o run --output-format csv -- python "$R0/tools/kbench.py" --no-multistream --rounds 2 --only "$V" > "$R0/gpurun_out/kp$i.log" 2>&1
  rc=$?; echo "== $V (rc=$rc)"; grep -v amdgpu.ids "$R0/gpurun_out/kp$i.log" | grep median; python "$R0/tools/kstats.py" "$R0/gpurun_out/kp$i/run_kernel_stats.csv" | grep -v rocclr
  [ $rc -ne 0 ] && exit $rc
done
exit 0
