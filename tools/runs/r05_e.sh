# round 5: compact group kernel beside a ring + its forced-parity tests, then the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_e
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_group_compact.py "tests/test_gpu_desc_multi.py::test_desc_multi_beside_running_ring" tests/test_gpu_ring.py > $O/tests_compact.log 2>&1 &&
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "rc=$?" >> $O/done.txt
