# iteration: membench ceilings, GPU parity tests, C2 kbench per group-scan mode
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 120 ./tools/membench > gpurun_out/membench.log 2>&1; rc=$?; cat gpurun_out/membench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for G in ${GSCAN:-2 1}; do
  echo "== NBG_GSCAN=$G"
  NBG_GSCAN=$G timeout -k 10 300 python tools/kbench.py --only "${ONLY:-full path,hist}" "$@" > gpurun_out/kbench_g$G.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/kbench_g$G.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
