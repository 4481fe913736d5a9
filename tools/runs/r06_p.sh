# round 6: drop-in thread placement A/B at 16 pipelines (dealt over the L3 caches of the GPU's socket, or
# packed on the first cores), 3 alternating rounds, plus 4 pipelines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_p
mkdir -p $O
timeout -k 10 500 python3 tools/dropin_bench.py --ab-spread > $O/ab.json 2> $O/ab.err
echo "rc=$?" >> $O/done.txt
# the CPU baseline under both placements (bench.py's cpu_baseline over its 8 C2 batches; no GPU)
grep -q "rc=0" $O/done.txt &&
timeout -k 10 300 python3 -c "
import json, sys
sys.path.insert(0, '.')
import bench, netbricks_amd as nb
bufs = [nb.make_trace(bench.BATCH, 0, seed=bench.shard_seed(0, b))[0] for b in range(bench.N_BATCHES)]
lut = nb.build_lut([f'backend-{i}' for i in range(bench.N_BACKENDS)], bench.TABLE)
print(json.dumps(bench.cpu_baseline(bufs, lut)))
" > $O/cpu_baseline.json 2> $O/cpu_baseline.err
echo "rc2=$?" >> $O/done.txt
