# round 5: the grouped ring's producer loop with pooled events (bench.py) vs one event created per
# burst (bench_prev.py = the previous commit's bench.py); ring variants only, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_w
mkdir -p $O
for r in 0 1; do
  for b in bench_prev bench; do
    NBG_BENCH_FULL=$O/full_${b}_$r.json timeout -k 10 300 python3 $b.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline --no-multi --no-imix --no-c4 > $O/${b}_$r.json 2> $O/${b}_$r.err || exit 1
  done
done
for b in bench_prev bench; do
  NBG_LIB_OVERRIDE=tools/ab/lib_gzero.so NBG_BENCH_FULL=$O/full_gzero_${b}.json timeout -k 10 300 python3 $b.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline --no-multi --no-imix --no-c4 > $O/gzero_${b}.json 2> $O/gzero_${b}.err || exit 1
done
echo "rc=$?" >> $O/done.txt
