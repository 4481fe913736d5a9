#!/bin/bash
# Round 3: does a longer warm-up raise the headline?  --warmup 5 / 100 / 400 (steps of 8 batches),
# headline only, multi (default) and launch paths, two passes.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
O=gpurun_out/r03_warm.txt
: > $O
for pass in 1 2; do
  for h in multi launch; do
    for W in 5 100 400; do
      timeout -k 10 300 python -u bench.py --headline $h --warmup $W --steps 50 --no-variants --no-pmc --no-cpu-baseline > gpurun_out/w.json 2> gpurun_out/w.err || { tail -3 gpurun_out/w.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('gpurun_out/w.json').read().strip().splitlines()[-1])
print('pass $pass $h warmup $W', d['value'], 'steady', d['steady_state']['value'], 'roof us', d['roofline']['avg_launch_us'])" >> $O
    done
  done
done
cat $O
