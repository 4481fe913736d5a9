#!/bin/bash
# Round 3: descriptor-ring replicas (NBG_RING_REPS: block b reads replica b % reps) against one copy,
# read only, producer in the loop (512 batches) and every batch posted ahead (60), three passes;
# then in place and the SPROBE build's counters at the default.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
O=gpurun_out/r03_ring_reps.txt
: > $O
for pass in 1 2 3; do
  for R in 1 64 256; do
    echo "== pass $pass reps $R loop" >> $O
    NBG_RING_REPS=$R timeout -k 10 120 tools/ring_bench ro 512 >> $O 2>&1 || exit 1
    echo "== pass $pass reps $R ahead" >> $O
    NBG_RING_REPS=$R timeout -k 10 120 tools/ring_bench ro 60 1048576 ahead >> $O 2>&1 || exit 1
  done
  echo "== pass $pass in place reps 64" >> $O
  timeout -k 10 120 tools/ring_bench ip 512 >> $O 2>&1 || exit 1
done
mkdir -p /tmp/ab_probe && ln -sf $PWD/tools/ab/lib_ringprobe.so /tmp/ab_probe/libnbgpu.so
echo "== probe loop reps 64" >> $O
LD_LIBRARY_PATH=/tmp/ab_probe timeout -k 10 120 tools/ring_bench ro 512 >> $O 2>&1 || exit 1
grep -v amdgpu.ids $O
