#!/bin/bash
# Round 3: where the ring's 1.5 us per unit step goes: default (write-through backend stores) against
# plain stores (abl1) and no backend stores (abl2), read only ahead / loop, in place loop; three
# interleaved passes; then per-block step times (SPROBE) ahead.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
O=gpurun_out/r03_ring_ab3.txt
: > $O
for b in ring_abl1 ring_abl2 ringprobe; do mkdir -p /tmp/ab_$b && ln -sf $PWD/tools/ab/lib_$b.so /tmp/ab_$b/libnbgpu.so; done
for pass in 1 2 3; do
  for b in default ring_abl1 ring_abl2; do
    L=""; [ $b != default ] && L=/tmp/ab_$b
    for m in "ro 60 1048576 ahead" "ro 512" "ip 512"; do
      echo "== pass $pass $b $m" >> $O
      LD_LIBRARY_PATH=$L timeout -k 10 120 tools/ring_bench $m >> $O 2>&1 || exit 1
    done
  done
done
echo "== probe ahead" >> $O
NBG_RING_PROBE_STEP=200 LD_LIBRARY_PATH=/tmp/ab_ringprobe timeout -k 10 120 tools/ring_bench ro 60 1048576 ahead >> $O 2>&1 || exit 1
grep -v amdgpu.ids $O | paste - - | sed 's/"n_pkts.*"launch_us"/ launch/; s/, "ring_wall[^,]*//; s/, "ring_gpps.*"ahead": [a-z]*//'
