#!/bin/bash
# Round 3: why the persistent ring runs slower than one launch per batch.  C++ producer (ring_bench,
# read only) against builds without write-through backend stores (abl1: plain stores, abl2: none)
# and without the page touches (nowarm); then the per-step timeline of the SPROBE build with every
# batch posted ahead (no producer in the loop).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
O=gpurun_out/r03_ring_diag.txt
: > $O
for b in ring_abl1 ring_abl2 ring_nowarm; do mkdir -p /tmp/ab_$b && ln -sf $PWD/tools/ab/lib_$b.so /tmp/ab_$b/libnbgpu.so; done
for pass in 1 2; do
  echo "== pass $pass default" >> $O
  timeout -k 10 120 tools/ring_bench ro 256 >> $O 2>&1 || exit 1
  for b in ring_abl1 ring_abl2 ring_nowarm; do
    echo "== pass $pass $b" >> $O
    LD_LIBRARY_PATH=/tmp/ab_$b timeout -k 10 120 tools/ring_bench ro 256 >> $O 2>&1 || exit 1
  done
done
echo "== timeline ringprobe" >> $O
NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_ringprobe.so NBG_RING_PROBE_STEP=24 timeout -k 10 300 python3 -u tools/ring_probe.py --variants none --batches 64 --timeline >> $O 2>&1 || exit 1
grep -v amdgpu.ids $O
