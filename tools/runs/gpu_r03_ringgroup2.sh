#!/bin/bash
# Round 3: ring grouping on several side streams: the ring tests, then the ring variants of the
# bench line with 1, 2 and 3 grouping streams.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ring.py > gpurun_out/r03_ringgroup_tests.txt 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r03_ringgroup_tests.txt | tail -3; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r03_ringgroup_tests.txt | head; exit $rc; }
for G in 1 2 3 4 2 3 4; do
  NBG_BENCH_RING_GROUP_STREAMS=$G timeout -k 10 300 python -u bench.py --no-imix --no-multi --no-pmc --no-cpu-baseline > gpurun_out/bench_g$G.json 2> gpurun_out/bench_g$G.err || { tail -3 gpurun_out/bench_g$G.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/bench_g$G.json').read().strip().splitlines()[-1])
v=d['variants']
print('G=$G', 'headline', d['value'], 'ring_ip', v['ring_in_place']['us_per_batch'], 'grouped', v['ring_in_place_grouped']['us_per_batch'], v['ring_in_place_grouped']['value'])
"
done
