# round 5: group kernel bin-width edge cases (tests/test_gpu_parity.py::test_group_bin_widths)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_u
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k group_bin_widths > $O/tests.log 2>&1
echo "rc=$?" >> $O/done.txt
