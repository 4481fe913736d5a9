#!/bin/bash
# Round 3, second session: the whole -m gpu suite + smoke on the restored tree, the ring against one
# launch per batch from the C++ producer (read only and in place), then the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
bash tools/gpu_suite.sh || exit $?
for v in ro ip; do
  timeout -k 10 120 tools/ring_bench $v 1024 > gpurun_out/ring_bench_$v.json 2> gpurun_out/ring_bench_$v.err || { cat gpurun_out/ring_bench_$v.err; exit 1; }
  cat gpurun_out/ring_bench_$v.json
done
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -3 gpurun_out/bench.err; cut -c1-1500 gpurun_out/bench.json; exit $rc
