# round 5: the grouped ring's gating cost split: gnone = gate kernel only, gzero = no gate and no launches
# (host bookkeeping and events only); ablation builds, timing only
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_v
mkdir -p $O
for r in 0 1; do
  for v in gnone gzero; do
    L=""; [ $v != tree ] && L=tools/ab/lib_$v.so
    NBG_LIB_OVERRIDE=$L NBG_BENCH_FULL=$O/full_${v}_$r.json timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline --no-multi --no-imix --no-c4 > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit 1
  done
done
echo "rc=$?" >> $O/done.txt
