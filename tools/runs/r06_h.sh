# host-batch server: its GPU tests, the host-path tests, then the drop-in sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_h
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_host_ring.py tests/test_gpu_pipeline.py tests/test_gpu_zerocopy.py > $O/tests.log 2>&1 &&
timeout -k 10 600 python3 tools/dropin_bench.py --extra > $O/dropin.json 2> $O/dropin.err
echo "rc=$?" >> $O/done.txt
