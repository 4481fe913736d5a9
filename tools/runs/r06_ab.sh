# round 6: the pipeline and host-ring GPU tests after the last test edits
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_ab
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pipeline.py tests/test_gpu_host_ring.py > $O/tests.log 2>&1
echo "rc=$?" >> $O/done.txt
