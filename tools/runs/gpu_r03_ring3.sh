#!/bin/bash
# Round 3: the ring kernel with a control wave (descriptor fetches out of the tile waves' vmcnt):
# parity, then tools/runs/gpu_r03_ring_ab.sh (C++ producer timing, store ablations, timeline).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ring.py > gpurun_out/r03_ring3_tests.txt 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r03_ring3_tests.txt | head -20; [ $rc -eq 0 ] || exit $rc
bash tools/runs/gpu_r03_ring_ab.sh
