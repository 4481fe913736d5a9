# A/B: run kbench against every tools/ab/lib_*.so, interleaved over 2 passes (same box, same buffers)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for pass in 1 2; do
  for L in tools/ab/lib_*.so; do
    echo "== $L (pass $pass)"
    NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 300 python tools/kbench.py "$@" > gpurun_out/ab.log 2>&1
    rc=$?; grep median gpurun_out/ab.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab.log; exit $rc; }
  done
done
exit 0
