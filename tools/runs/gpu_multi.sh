# Multi-batch launch: its parity tests, then kbench A/B (single-batch kernels of HEAD vs the
# working tree, and the working tree's multi-batch calls), two passes.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_multi.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_multi.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/pytest_multi.log | head -20; exit $rc; }
for pass in 1 2; do
  for L in tools/ab/lib_*.so; do
    echo "== $L (pass $pass)"
    ONLY="classify noswap hist,full path inplace,full path mac_out"
    case $L in *multi*) ONLY="$ONLY,multi";; esac
    NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 300 python -u tools/kbench.py --no-multistream --rounds 5 --only "$ONLY" > gpurun_out/ab.log 2>&1
    rc=$?; grep median gpurun_out/ab.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab.log; exit $rc; }
  done
done
