#!/bin/bash
# Round 3: the ring's variance.  The C++ producer (ring_bench) with the producer in the loop (512
# batches) and with every batch posted ahead (60 batches), default build and the SPROBE build (ring
# kernel counters: prefetches, batches taken, empty prefetches, idle entries per block).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
O=gpurun_out/r03_ring_diag2.txt
: > $O
mkdir -p /tmp/ab_probe && ln -sf $PWD/tools/ab/lib_ringprobe.so /tmp/ab_probe/libnbgpu.so
for pass in 1 2 3; do
  echo "== pass $pass default loop" >> $O
  timeout -k 10 120 tools/ring_bench ro 512 >> $O 2>&1 || exit 1
  echo "== pass $pass default ahead" >> $O
  timeout -k 10 120 tools/ring_bench ro 60 1048576 ahead >> $O 2>&1 || exit 1
  echo "== pass $pass probe loop" >> $O
  LD_LIBRARY_PATH=/tmp/ab_probe timeout -k 10 120 tools/ring_bench ro 512 >> $O 2>&1 || exit 1
  echo "== pass $pass probe ahead" >> $O
  LD_LIBRARY_PATH=/tmp/ab_probe timeout -k 10 120 tools/ring_bench ro 60 1048576 ahead >> $O 2>&1 || exit 1
done
grep -v amdgpu.ids $O
