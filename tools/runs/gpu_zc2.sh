cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_zerocopy.py > gpurun_out/zc_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/zc_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/e2e_bench.py > gpurun_out/e2e.json 2> gpurun_out/e2e.err
rc=$?; cat gpurun_out/e2e.json; [ $rc -ne 0 ] && tail -5 gpurun_out/e2e.err; exit $rc
