# A/B over tools/ab/lib_*.so in one GPU call: GPU parity of the builds named in $TEST_LIBS, then
# kbench passes interleaved across builds, with the L2-gathered and the LDS-staged LUT.
# Extra args go to kbench.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for L in $TEST_LIBS; do
  NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_$L.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -x \
    -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$L.log 2>&1
  rc=$?; echo "pytest($L) rc=$rc"; tail -2 gpurun_out/pytest_gpu_$L.log; [ $rc -ne 0 ] && exit $rc
done
for pass in 1 2; do
  for LDS in "" "--lut-lds"; do
    for L in tools/ab/lib_*.so; do
      echo "== $L $LDS (pass $pass)"
      NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 300 python -u tools/kbench.py $LDS "$@" > gpurun_out/ab.log 2>&1
      rc=$?; grep median gpurun_out/ab.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab.log; exit $rc; }
    done
  done
done
exit 0
