# A/B over every tools/ab/lib_*.so: GPU parity of each, then kbench (2 passes)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for L in tools/ab/lib_*.so; do
  NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest($L) rc=$rc"; tail -1 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
done
for pass in 1 2; do
  for L in tools/ab/lib_*.so; do
    echo "== $L (pass $pass)"
    NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 300 python tools/kbench.py "$@" > gpurun_out/ab.log 2>&1
    rc=$?; grep median gpurun_out/ab.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab.log; exit $rc; }
  done
done
exit 0
