#!/bin/bash
# Round 3: lag kernel after the slow-path fix: parity of the streaming kernels, ablation timings,
# and the per-wave timelines.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lag.py tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_fuzz.py > gpurun_out/r03c_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03c_tests.log; exit 1; }
tail -2 gpurun_out/r03c_tests.log
bash tools/runs/gpu_lag_abl.sh || exit 1
bash tools/runs/gpu_r03_tl.sh > /dev/null 2>&1; grep -E "==|interval|prologue|exit  " gpurun_out/r03_tl_group.txt gpurun_out/r03_tl_lag.txt
