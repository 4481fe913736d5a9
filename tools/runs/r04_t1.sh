set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ring.py tests/test_gpu_parity.py tests/test_gpu_multi.py > gpurun_out/r04_t1.log 2>&1
echo "rc=$?" >> gpurun_out/r04_t1.log
