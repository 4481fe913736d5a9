# rocprof of bench.py --multi-only per tools/ab/lib_*.so (the last 50 launches of each classify
# kernel = the single-stream kernel pass), two passes.
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mab
for pass in 1 2; do
  for L in "$R0"/tools/ab/lib_*.so; do
    n=$(basename "$L" .so)
    echo "== $n (pass $pass)"
    ( cd /tmp && export TMPDIR=/tmp && NBG_LIB_OVERRIDE=$L timeout -k 10 300 rocprofv3 --kernel-trace -d "$R0/gpurun_out/mab/${n}_$pass" -o run --output-format csv -- python "$R0/bench.py" --inline --no-pmc --no-cpu-baseline --multi-only --steps 200 > "$R0/gpurun_out/mab/${n}_$pass.json" 2> "$R0/gpurun_out/mab/${n}_$pass.err" )
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc"; tail -5 "$R0/gpurun_out/mab/${n}_$pass.err"; exit $rc; }
    python "$R0/tools/ktrace_last.py" "$R0/gpurun_out/mab/${n}_$pass/run_kernel_trace.csv" 50 | grep -v rocclr
  done
done
