#!/bin/bash
# Round 3: nbg_ring_group parity (grouping launches beside the resident ring kernel) and the ring tests.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ring.py > gpurun_out/r03_ringgroup_tests.txt 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed|assert" gpurun_out/r03_ringgroup_tests.txt | tail -20; exit $rc
