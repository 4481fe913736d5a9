# round 5: group-kernel A/B through the whole bench, twice each (committed kernel / prologue
# overlapped with the first chunk's ranks / wave-segment direct stores)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_d
mkdir -p $O
for r in 0 1; do for v in oldgroup overlap newgroup; do
  NBG_BENCH_FULL=$O/full_${v}_$r.json NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_$v.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit 1
done; done
echo "rc=$?" >> $O/done2.txt
