#!/bin/bash
# Round 3: ring kernel variants with the relay: default (2 LDS tiles per wave), NBG_SRING=3 (3 tiles
# per wave: read only only, in place does not fit LDS), NBG_RING_WARM=0 (no page touches ahead of a
# batch); read only (loop / ahead) and in place (loop), three interleaved passes.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
O=gpurun_out/r03_ring_ab2.txt
: > $O
for b in ring_s3 ring_nowarm; do mkdir -p /tmp/ab_$b && ln -sf $PWD/tools/ab/lib_$b.so /tmp/ab_$b/libnbgpu.so; done
for pass in 1 2 3; do
  for b in default ring_s3 ring_nowarm; do
    L=""; [ $b != default ] && L=/tmp/ab_$b
    for m in "ro 512" "ro 60 1048576 ahead" "ip 512"; do
      [ $b = ring_s3 ] && [ "${m:0:2}" = ip ] && continue
      echo "== pass $pass $b $m" >> $O
      LD_LIBRARY_PATH=$L timeout -k 10 120 tools/ring_bench $m >> $O 2>&1 || exit 1
    done
  done
done
grep -v amdgpu.ids $O | paste - - | sed 's/"n_pkts.*"launch_us"/ launch/; s/, "ring_wall.*//' 
