# C3 with the scan folded into the group kernel's prologue (NBG_GSCAN=2: every group block sums the
# partition rows itself, no scan_kernel launch) against scan_kernel (default), after parity.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
NBG_GSCAN=2 timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "c3_full or imix_descriptors" > gpurun_out/scan_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/scan_pytest.log; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for g in 0 2; do
    for v in in_place read_only; do
      echo "== NBG_GSCAN=$g $v"
      NBG_GSCAN=$g timeout -k 10 200 python -u tools/config_bench.py --config c3 --c3-variant $v > gpurun_out/cs.json 2> gpurun_out/cs.err || { tail -3 gpurun_out/cs.err; exit 1; }
      cat gpurun_out/cs.json
    done
  done
done
exit 0
