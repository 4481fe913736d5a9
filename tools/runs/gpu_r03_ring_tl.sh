#!/bin/bash
# Round 3: per-block step times of the ring kernel (SPROBE build) in fast and slow runs: 16 unit
# steps from step 2000 (loop, 512 batches) or 200 (ahead, 60 batches), six runs each.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
O=gpurun_out/r03_ring_tl.txt
: > $O
mkdir -p /tmp/ab_probe && ln -sf $PWD/tools/ab/lib_ringprobe.so /tmp/ab_probe/libnbgpu.so
for pass in 1 2 3 4 5 6; do
  echo "== pass $pass loop" >> $O
  NBG_RING_PROBE_STEP=2000 LD_LIBRARY_PATH=/tmp/ab_probe timeout -k 10 120 tools/ring_bench ro 512 >> $O 2>&1 || exit 1
  echo "== pass $pass ahead" >> $O
  NBG_RING_PROBE_STEP=200 LD_LIBRARY_PATH=/tmp/ab_probe timeout -k 10 120 tools/ring_bench ro 60 1048576 ahead >> $O 2>&1 || exit 1
done
grep -v amdgpu.ids $O
