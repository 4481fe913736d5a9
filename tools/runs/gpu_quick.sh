# quick GPU iteration: parity tests, variant micro-benchmark per NBG_ROUNDS, rocprof kernel trace
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for R in ${ROUNDS:-1}; do
  echo "== NBG_ROUNDS=$R"
  NBG_ROUNDS=$R timeout -k 10 300 python tools/kbench.py "$@" > gpurun_out/kbench_r$R.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/kbench_r$R.log; [ $rc -ne 0 ] && exit $rc
done
R0="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
NBG_ROUNDS=${PROF_ROUNDS:-1} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R0/gpurun_out/kprof" -o run --output-format csv -- python "$R0/tools/kbench.py" --rounds 1 "$@" > "$R0/gpurun_out/kprof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; python "$R0/tools/kstats.py" "$R0/gpurun_out/kprof/run_kernel_stats.csv"
exit $rc
