#!/bin/bash
# Round 3: partition histograms written by the ring kernel (nbg_ring_group = one group launch):
# the ring tests, the ring C++ timing (does the flush slow the ring?), then the bench line.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ring.py > gpurun_out/r03_ringhist_tests.txt 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r03_ringhist_tests.txt | tail -2; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert|Mismatch" gpurun_out/r03_ringhist_tests.txt | head; exit $rc; }
for v in ro ip; do timeout -k 10 120 tools/ring_bench $v 1024 || exit 1; done
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -3 gpurun_out/bench.err; exit $rc
