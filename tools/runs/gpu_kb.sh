# parity tests + kbench (single stream + multistream) for quick A/B of kernel changes
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/kbench.py "$@" > gpurun_out/kb.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/kb.log; exit $rc
