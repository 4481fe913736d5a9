#!/bin/bash
# Round 3: the persistent RX ring (nbg_ring_*) parity and timing, and the multi-launch graph capture
# (captured zeroing as a kernel node) against direct calls on torch's null stream.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
O=gpurun_out/r03_ring.txt
: > $O
run() { echo "== $*" | tee -a $O; "$@" >> $O 2>&1; local rc=$?; echo "rc=$rc" | tee -a $O; return $rc; }
run timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ring.py &&
run timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_graph.py &&
run timeout -k 10 300 python3 -u tools/ring_probe.py &&
run env NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_ringprobe.so NBG_RING_PROBE_STEP=24 timeout -k 10 300 python3 -u tools/ring_probe.py --batches 64 --timeline
echo "exit $?"; grep -v amdgpu.ids $O | grep -E "PASS|FAIL|Error|error|rc=|==|\{" | cut -c1-400
