#!/bin/bash
# Round 3: the ring's per-batch time by producer pattern (one post per completion, 32-slot refills,
# everything posted ahead) and over the run (slope per eighth), read only and in place, 2 passes.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
O=gpurun_out/r03_ring_modes.txt
: > $O
for pass in 1 2; do
  for m in "ro 1024" "ro 1024 1048576 chunk" "ro 60 1048576 ahead" "ip 1024" "ip 1024 1048576 chunk" "ip 60 1048576 ahead"; do
    echo "== pass $pass $m" >> $O
    timeout -k 10 120 tools/ring_bench $m >> $O 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O | paste - - | sed 's/"n_pkts.*"launch_us"/ launch/; s/, "ring_wall[^,]*//; s/, "ring_gpps.*"ahead": [a-z]*//'
