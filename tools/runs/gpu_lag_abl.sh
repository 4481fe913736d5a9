#!/bin/bash
# Round 3: cost of the lagged-grouping launch, by ablation build (NBG_LAG_ABL: 1 no prologue, 2 no
# pieces in the unit loop, 3 neither, 4 no perm stores), two interleaved passes, one process per build.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
O=gpurun_out/r03_lag_abl.txt
: > $O
for pass in 1 2; do
  for v in 0 1 2; do
    NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_lagabl$v.so timeout -k 10 120 python3 tools/lag_probe.py >> $O 2>> gpurun_out/r03_lag_abl.err || { echo "probe $v failed"; tail -5 gpurun_out/r03_lag_abl.err; exit 1; }
  done
done
cat $O
