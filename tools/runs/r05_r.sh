# round 5: group kernels at 6 / 8 waves per SIMD (tools/ab/lib_gw6.so / lib_gw8.so: launch bounds only,
# spills) against the tree (4): the group launches alone and the bench's multi-batch paths, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_r
mkdir -p $O
for r in 0 1; do
  for v in tree gw6 gw8; do
    L=""; [ $v != tree ] && L=tools/ab/lib_$v.so
    NBG_LIB_OVERRIDE=$L timeout -k 10 120 python3 tools/group_kbench.py --label $v >> $O/kbench.txt 2>> $O/kbench.err || exit 1
    NBG_LIB_OVERRIDE=$L NBG_BENCH_FULL=$O/full_${v}_$r.json timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline --no-ring --no-c4 > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit 1
  done
done
echo "rc=$?" >> $O/done.txt
