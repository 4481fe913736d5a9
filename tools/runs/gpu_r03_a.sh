#!/bin/bash
# Round 3, first GPU pass: the new lagged-grouping and C4-shard parity tests, then the whole GPU
# suite, then the driver's bench command and a kernel-trace profile of it.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lag.py tests/test_gpu_c4_shards.py > gpurun_out/r03a_new_tests.log 2>&1 || { echo "new tests failed"; tail -40 gpurun_out/r03a_new_tests.log; exit 1; }
tail -3 gpurun_out/r03a_new_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/r03a_gpu_tests.log 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/r03a_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03a_gpu_tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err || { echo "bench failed"; tail -30 gpurun_out/r03a_bench.err; exit 1; }
cat gpurun_out/r03a_bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r03a_prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --inline --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/r03a_prof_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r03a_prof.err" || { echo "profile failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/r03a_prof.err"; exit 1; }
echo done
