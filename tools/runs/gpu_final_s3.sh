# Session-3 measurement set: GPU suite + smoke, default bench, rocprof (single-stream variants,
# multi-batch kernel pass), PMC-free; then C3/C5 with and without nt packet loads in the
# tile-per-wave kernel (config_bench, 3 streams).
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"
bash tools/gpu_suite.sh || exit $?
bash tools/runs/gpu_bench_multi.sh || exit $?
python tools/ktrace_last.py gpurun_out/prof/multi/run_kernel_trace.csv 50
cd "$R0"
for L in tools/ab/lib_*.so; do
  NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 300 python tools/config_bench.py --steps 200 --warmup 20 --streams 3 > gpurun_out/cfg_$(basename $L .so).json 2> gpurun_out/cfg.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/cfg.err; exit $rc; }
  echo "== $L"; cat gpurun_out/cfg_$(basename $L .so).json
done
timeout -k 10 300 python -u tools/config_bench.py --cpu-baseline > gpurun_out/configs.json 2> gpurun_out/configs.err
rc=$?; cat gpurun_out/configs.json; exit $rc
