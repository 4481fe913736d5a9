#!/bin/bash
# Round 3: the multi-batch headline by batches per launch (K) and streams (S), two passes, bench
# headline only (--no-variants --no-pmc --no-cpu-baseline).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
O=gpurun_out/r03_multi_sweep.txt
: > $O
for pass in 1 2; do
  for ks in "4 2" "4 3" "8 2" "2 3" "2 2"; do
    set -- $ks
    NBG_BENCH_MULTI_K=$1 NBG_BENCH_MULTI_STREAMS=$2 timeout -k 10 300 python -u bench.py --no-variants --no-pmc --no-cpu-baseline > gpurun_out/ms.json 2> gpurun_out/ms.err || { tail -3 gpurun_out/ms.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/ms.json').read().strip().splitlines()[-1])
print('pass $pass K=$1 S=$2', d['value'], d['steady_state']['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])" >> $O
  done
done
cat $O
