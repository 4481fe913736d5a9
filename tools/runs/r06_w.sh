# round 6: the 32-B staged windows and lengths written with non-temporal stores (this tree) against plain
# stores (NBG_HOST_NT=0), drop-in at 16 and 1 pipelines, 3 alternating rounds on one box; then the GPU
# tests of the host path
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_w
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_host_ring.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_zerocopy.py > $O/tests.log 2>&1 &&
timeout -k 10 600 python3 tools/dropin_bench.py --ab-env NBG_HOST_NT=0 > $O/ab.json 2> $O/ab.err
echo "rc=$?" >> $O/done.txt
