# Dynamic unit assignment (a_dyn) vs static interleave (b_static): parity of the C2 tests under the
# new default build first, then kbench passes over both builds.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "c2 or multi_chunk or no_swap or mac_out or repeat" > gpurun_out/dyn_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/dyn_pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/runs/gpu_ab_seq.sh
