#!/bin/bash
# Round 3: the ring with the relay kernel (no classify CU reads host memory): parity tests, then the
# C++ producer read only / in place, loop and posted ahead, three passes.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
O=gpurun_out/r03_relay.txt
: > $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ring.py > gpurun_out/r03_relay_tests.txt 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r03_relay_tests.txt | tail -12; [ $rc -eq 0 ] || exit $rc
for pass in 1 2 3; do
  for v in ro ip; do
    echo "== pass $pass $v loop" >> $O
    timeout -k 10 120 tools/ring_bench $v 512 >> $O 2>&1 || exit 1
    echo "== pass $pass $v ahead" >> $O
    timeout -k 10 120 tools/ring_bench $v 60 1048576 ahead >> $O 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O
