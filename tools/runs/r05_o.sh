# round 5: C3 / C5 with 16 IMIX batches per launch against 8 (NBG_BENCH_IMIX_MULTI_K), whole bench, twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_o
mkdir -p $O
for r in 0 1; do for k in 16 8; do
  NBG_BENCH_IMIX_MULTI_K=$k NBG_BENCH_FULL=$O/full_k${k}_$r.json timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline --no-ring > $O/bench_k${k}_$r.json 2> $O/bench_k${k}_$r.err || exit 1
done; done
echo "rc=$?" >> $O/done.txt
for b in 4 8 2; do
  NBG_BENCH_RING_GROUP_BURST=$b NBG_BENCH_FULL=$O/full_burst${b}.json timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline --no-imix > $O/bench_burst${b}.json 2> $O/bench_burst${b}.err || exit 1
done
echo "rc_burst=$?" >> $O/done.txt
