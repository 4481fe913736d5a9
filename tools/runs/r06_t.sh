# round 6: C3's partition rows from the classify kernel's flush (NBG_HIST_KERNEL_BINS=2000: 1001 bins
# under the threshold) against hist_kernel (default), two alternating rounds of bench.py's variants
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_t
mkdir -p $O
F="--steps 5 --warmup 2 --no-ring --no-c4 --no-pmc --no-e2e --no-cpu-baseline"
for r in 0 1; do
  NBG_BENCH_FULL=$O/base_$r.json timeout -k 10 300 python3 bench.py $F > $O/base_$r.line 2> $O/base_$r.err &&
  NBG_HIST_KERNEL_BINS=2000 NBG_BENCH_FULL=$O/flush_$r.json timeout -k 10 300 python3 bench.py $F > $O/flush_$r.line 2> $O/flush_$r.err || break
done
echo "rc=$?" >> $O/done.txt
