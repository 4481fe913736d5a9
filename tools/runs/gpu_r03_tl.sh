#!/bin/bash
# Round 3: per-wave timeline of the streaming launch with separate grouping vs lagged grouping.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_sprobe.so
timeout -k 10 120 python3 tools/sprobe.py --group > gpurun_out/r03_tl_group.txt 2>&1 && \
timeout -k 10 120 python3 tools/sprobe.py --lag > gpurun_out/r03_tl_lag.txt 2>&1
rc=$?; grep -E "==|interval|prologue|step4|exit  |tile 4" gpurun_out/r03_tl_group.txt gpurun_out/r03_tl_lag.txt; exit $rc
