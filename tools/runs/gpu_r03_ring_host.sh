#!/bin/bash
# Round 3: the ring with the producer's stream queries throttled (nbgpu_api.hip ring_gone): C++
# producer, read only and in place, four passes each, against one launch per batch.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
O=gpurun_out/r03_ring_host.txt
: > $O
for pass in 1 2 3 4; do
  for v in ro ip; do
    echo "== pass $pass $v" >> $O
    timeout -k 10 120 tools/ring_bench $v 512 >> $O 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O
