#!/bin/bash
# Round 3: the streaming kernel's in-place window stores write-through (sc1, NBG_STREAM_WT=1) against
# nt (default): bench headline (4 x 1M per launch) and the launch-per-batch variant, two passes.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
O=gpurun_out/r03_stream_wt.txt
: > $O
for pass in 1 2; do
  for L in default stream_wt; do
    E=""; [ $L != default ] && E="NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_$L.so"
    env $E timeout -k 10 300 python -u bench.py --no-pmc --no-cpu-baseline --no-imix --no-ring > gpurun_out/wt.json 2> gpurun_out/wt.err || { tail -3 gpurun_out/wt.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/wt.json').read().strip().splitlines()[-1]); v=d['variants']
print('pass $pass $L headline', d['value'], 'steady', d['steady_state']['value'], 'multi launch us', d['roofline']['avg_launch_us'],
      '| launch_in_place', v['launch_in_place']['value'], v['launch_in_place']['avg_launch_us'], '| records', v['records']['avg_launch_us'], '| c4', v['c4_shard']['avg_launch_us'])" >> $O
  done
done
cat $O
