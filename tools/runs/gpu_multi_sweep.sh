# multi-batch variants by (batches per launch, streams): whole-job rate and the kernel pass
cd "$GRAFT_REPO_ROOT" || exit 9
for kv in "4 2" "2 3" "2 2" "8 1" "4 1"; do
  set -- $kv
  NBG_BENCH_MULTI_K=$1 NBG_BENCH_MULTI_STREAMS=$2 timeout -k 10 200 python bench.py --inline --no-pmc --no-cpu-baseline --multi-only --steps 400 > gpurun_out/sw.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/sw.json'))
for k,v in d.items(): print('K=$1 streams=$2', k, 'value', v['value'], 'launch_us', v['avg_launch_us'], 'frac', v['frac'])"
done
