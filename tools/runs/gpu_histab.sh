# hist-kernel vs classify-histogram A/B for C3 (1001 bins) and C2 (66 bins)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for H in 257 100000; do
  echo "== C3 NBG_HIST_KERNEL_BINS=$H"
  NBG_HIST_KERNEL_BINS=$H timeout -k 10 300 python tools/config_bench.py --config c3 > gpurun_out/c3h.json 2>/dev/null
  rc=$?; cat gpurun_out/c3h.json; [ $rc -ne 0 ] && exit $rc
done
for H in 257 2; do
  echo "== C2 NBG_HIST_KERNEL_BINS=$H"
  NBG_HIST_KERNEL_BINS=$H timeout -k 10 300 python tools/kbench.py --only "full path,x2 streams" --rounds 3 > gpurun_out/c2h.log 2>&1
  rc=$?; grep median gpurun_out/c2h.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
