# bench value (C2 in place + grouping, 3 streams) and the classify kernel pass: streaming kernel
# (default) vs the tile-per-wave kernel (NBG_STREAM=0), three interleaved passes
cd "$GRAFT_REPO_ROOT" || exit 9
for pass in 1 2 3; do
  for S in 1 0; do
    NBG_STREAM=$S timeout -k 10 300 python bench.py --inline --no-pmc --no-cpu-baseline --no-multi > gpurun_out/s.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/s.json')); r=d['roofline']; v=d['variants']
print('pass $pass NBG_STREAM=$S value', d['value'], 'classify_us', r['avg_launch_us'], '| records', v['records']['value'], v['records']['avg_launch_us'], '| read_only', v['read_only']['value'], v['read_only']['avg_launch_us'])"
  done
done
