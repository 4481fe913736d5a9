# A/B over libraries x NBG_TPW values (same box): kbench variants
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_new.so timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest(new) rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for cfg in ${CFGS:-old:1 new:1}; do
    L=${cfg%%:*}; T=${cfg##*:}
    echo "== lib_$L TPW=$T (pass $pass)"
    NBG_TPW=$T NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_$L.so timeout -k 10 300 python tools/kbench.py "$@" > gpurun_out/ab.log 2>&1
    rc=$?; grep median gpurun_out/ab.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab.log; exit $rc; }
  done
done
exit 0
