#!/bin/bash
# Round 3: lag-kernel parity (new tests) then the ablation timings.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lag.py tests/test_gpu_c4_shards.py tests/test_gpu_parity.py > gpurun_out/r03b_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03b_tests.log; exit 1; }
tail -2 gpurun_out/r03b_tests.log
bash tools/runs/gpu_lag_abl.sh
