#!/bin/bash
# Round 3: the ring tests (buffers reused across starts) and the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ring.py > gpurun_out/r03_check_tests.txt 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r03_check_tests.txt | tail -2; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r03_check_tests.txt | head; exit $rc; }
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -3 gpurun_out/bench.err; exit $rc
