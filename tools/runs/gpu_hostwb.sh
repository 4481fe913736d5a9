# Host-path MAC write-back with non-temporal stores (a_nt, default) against cached memcpy
# (b_cached): host-path parity with the default build, then tools/host_probe.py with each build.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py -k "host or pipeline or lemmy or c1" > gpurun_out/hwb_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/hwb_pytest.log; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for L in a_nt b_cached; do
    echo "== $L (pass $pass)"
    NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_$L.so timeout -k 10 300 python -u tools/host_probe.py > gpurun_out/hp.json 2> gpurun_out/hp.err || { tail -3 gpurun_out/hp.err; exit 1; }
    grep "room" gpurun_out/hp.err
  done
done
exit 0
