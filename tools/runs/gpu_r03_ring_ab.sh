#!/bin/bash
# Round 3: the ring against one launch per batch from a C++ producer (tools/ring_bench): with and
# without the control wave's page touches ahead of each batch (NBG_RING_WARM), three interleaved
# passes, one process per build (LD_LIBRARY_PATH puts the build's libnbgpu.so first); then the
# per-wave timelines of both (SPROBE builds).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
O=gpurun_out/r03_ring_ab.txt
: > $O
B="warm nowarm"
for b in $B; do mkdir -p /tmp/ab_$b && ln -sf $PWD/tools/ab/lib_ring_$b.so /tmp/ab_$b/libnbgpu.so; done
for pass in 1 2 3; do
  for b in $B; do
    for v in ro ip; do
      echo "== pass $pass $b $v" >> $O
      LD_LIBRARY_PATH=/tmp/ab_$b timeout -k 10 120 tools/ring_bench $v 512 >> $O 2>&1 || exit 1
    done
  done
done
for p in ringprobe ringprobe_nowarm; do
  echo "== timeline $p" >> $O
  NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_$p.so NBG_RING_PROBE_STEP=24 timeout -k 10 300 python3 -u tools/ring_probe.py --variants none --batches 64 --timeline 2>&1 | grep -v amdgpu.ids | tail -2 | head -1 >> $O || exit 1
done
cat $O
