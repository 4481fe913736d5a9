# NBG_STREAM_DESC (descriptor streaming kernel): its parity tests, the default-path C3/C5 parity
# tests, then config_bench C3/C5 with and without --stream-desc, on 1 and 3 streams, two passes.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_gpu_stream_desc.py "tests/test_gpu_parity.py::test_c3_full_1m" tests/test_gpu_lpm.py \
  tests/test_gpu_parity.py::test_imix_descriptors > gpurun_out/desc_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/desc_pytest.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/desc_ab.txt; : > $out
for pass in 1 2; do
  for S in 1 3; do
    for D in "" "--stream-desc"; do
      echo "== streams=$S ${D:-tile-per-wave} (pass $pass)" | tee -a $out
      timeout -k 10 300 python -u tools/config_bench.py --config c3,c5 --streams $S $D > gpurun_out/desc_ab.log 2>&1
      rc=$?; grep '^{' gpurun_out/desc_ab.log | tee -a $out; [ $rc -ne 0 ] && { tail -5 gpurun_out/desc_ab.log; exit $rc; }
    done
  done
done
exit 0
