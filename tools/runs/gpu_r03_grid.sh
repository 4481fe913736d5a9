#!/bin/bash
# Round 3: streaming-classify blocks per launch (NBG_STREAM_GRID): 256 (one per CU) against 255 / 248
# (the ring runs 255 classify blocks and rewrites faster): headline (4 x 1M per launch) and the
# launch-per-batch variant, two passes.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
O=gpurun_out/r03_grid.txt
: > $O
for pass in 1 2; do
  for G in 256 255 248; do
    NBG_STREAM_GRID=$G timeout -k 10 300 python -u bench.py --no-pmc --no-cpu-baseline --no-imix --no-ring > gpurun_out/g.json 2> gpurun_out/g.err || { tail -3 gpurun_out/g.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/g.json').read().strip().splitlines()[-1]); v=d['variants']
print('pass $pass grid $G headline', d['value'], 'multi launch us', d['roofline']['avg_launch_us'], '| launch_in_place', v['launch_in_place']['value'], v['launch_in_place']['avg_launch_us'], '| ro', v['read_only']['avg_launch_us'], '| ro multi4', v['read_only_multi4']['avg_launch_us'])" >> $O
  done
done
cat $O
