# kbench passes interleaved across tools/ab/lib_*.so (+ the tile-per-wave kernel, NBG_STREAM=0, of
# the first build) in one GPU call.  Extra args go to kbench.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
libs=$(ls tools/ab/lib_*.so)
first=$(echo $libs | cut -d' ' -f1)
for pass in 1 2; do
  echo "== tile-per-wave (NBG_STREAM=0) (pass $pass)"
  NBG_STREAM=0 NBG_LIB_OVERRIDE=$PWD/$first timeout -k 10 300 python -u tools/kbench.py "$@" > gpurun_out/ab.log 2>&1
  rc=$?; grep median gpurun_out/ab.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab.log; exit $rc; }
  for L in $libs; do
    echo "== $L (pass $pass)"
    NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 300 python -u tools/kbench.py "$@" > gpurun_out/ab.log 2>&1
    rc=$?; grep median gpurun_out/ab.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab.log; exit $rc; }
  done
done
exit 0
