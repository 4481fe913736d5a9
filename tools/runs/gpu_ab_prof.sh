# rocprofv3 kernel stats of bench.py's single-stream pass (all three C2 variants, grouping deferred)
# for every tools/ab/lib_*.so, two interleaved passes.  Then the default 3-stream bench per lib.
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abprof
for pass in 1 2; do
  for L in "$R0"/tools/ab/lib_*.so; do
    n=$(basename "$L" .so)
    echo "== $n (pass $pass)"
    ( cd /tmp && export TMPDIR=/tmp && NBG_LIB_OVERRIDE=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R0/gpurun_out/abprof/${n}_$pass" -o run --output-format csv -- python "$R0/bench.py" --inline --no-pmc --no-cpu-baseline --streams 1 --steps 200 --warmup 20 > "$R0/gpurun_out/abprof/${n}_$pass.json" 2> "$R0/gpurun_out/abprof/${n}_$pass.err" )
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc"; tail -5 "$R0/gpurun_out/abprof/${n}_$pass.err"; exit $rc; }
    python "$R0/tools/kstats.py" "$R0/gpurun_out/abprof/${n}_$pass/run_kernel_stats.csv" | grep classify_stream
  done
done
for L in "$R0"/tools/ab/lib_*.so; do
  n=$(basename "$L" .so)
  NBG_LIB_OVERRIDE=$L timeout -k 10 300 python "$R0/bench.py" --inline --no-pmc --no-cpu-baseline > "$R0/gpurun_out/abprof/${n}_bench.json" 2>&1 || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'value', d['value'], {k: v['value'] for k, v in d['variants'].items()})" "$R0/gpurun_out/abprof/${n}_bench.json" "$n"
done
