# round 4: C3 / C5 at 8 batches per launch with each handle's grouping on a low-priority stream and
# its classify on a high-priority one, against the same-stream default (same run)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_prio
mkdir -p $O
NBG_BENCH_IMIX_PRIO=1 timeout -k 10 600 python3 bench.py --no-ring --no-c4 --no-pmc --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "rc=$?" >> $O/done.txt
