# Group-kernel change: GPU parity (working tree), group phase probe, then kbench A/B of
# tools/ab/lib_*.so on the full path (C2 single + 4 streams, and C3-shaped IMIX / 1000 bins).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
NBG_LIB_OVERRIDE=$PWD/tools/abx/lib_gprobe.so timeout -k 10 120 python tools/gprobe_run.py > gpurun_out/gprobe.log 2>&1
rc=$?; grep GPROBE gpurun_out/gprobe.log | tail -3; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for L in tools/ab/lib_*.so; do
    echo "== $L C2 (pass $pass)"
    NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 300 python -u tools/kbench.py --rounds 3 --streams 2,4 \
      --only "full path inplace,full path mac_out,classify inplace hist,streams" > gpurun_out/ab.log 2>&1
    rc=$?; grep median gpurun_out/ab.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab.log; exit $rc; }
    echo "== $L C3 (pass $pass)"
    NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 300 python -u tools/kbench.py --mode 1 --nb 1000 --m 655373 --rounds 3 \
      --streams 4 --only "full path inplace,x4 streams" > gpurun_out/ab.log 2>&1
    rc=$?; grep median gpurun_out/ab.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab.log; exit $rc; }
  done
done
exit 0
