#!/bin/bash
# Round 3: the multi-batch deferred-group test, a single-stream kernel-trace profile of the bench's
# C2 headline launches (so rocprof's classify average is the single-launch duration the bench's
# events report), then the graph-replay root-cause probes (last: they capture multi-launch batches).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_multi.py > gpurun_out/r03e_multi.log 2>&1 || { echo "multi tests failed"; tail -30 gpurun_out/r03e_multi.log; exit 1; }
tail -2 gpurun_out/r03e_multi.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r03e_prof1" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --inline --streams 1 --steps 20 --warmup 5 --steady-steps 0 --no-variants --no-pmc --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/r03e_prof1_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r03e_prof1.err" || { echo "profile failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/r03e_prof1.err"; exit 1; }
cd "$GRAFT_REPO_ROOT" && cat gpurun_out/r03e_prof1_bench.json | head -c 600; echo
bash tools/runs/gpu_graph_rootcause.sh
