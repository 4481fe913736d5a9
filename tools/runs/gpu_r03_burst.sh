#!/bin/bash
# Round 3: ring burst posts (parity), then the default bench line (ring variants with burst posts).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ring.py > gpurun_out/r03_burst_tests.txt 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r03_burst_tests.txt | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -3 gpurun_out/bench.err; exit $rc
