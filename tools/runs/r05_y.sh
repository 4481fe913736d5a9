# round 5: the multi-batch streaming classify with write-through (sc1) window stores, as the ring's,
# instead of nt stores (tools/ab/lib_wt.so); bench --multi-only, alternating with the tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_y2
mkdir -p $O
for r in 0 1 2; do
  for v in tree wt; do
    L=""; [ $v != tree ] && L=tools/ab/lib_$v.so
    NBG_LIB_OVERRIDE=$L NBG_BENCH_FULL=$O/full_${v}_$r.json timeout -k 10 200 python3 bench.py --multi-only --steps 50 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline >> $O/$v.jsonl 2>> $O/$v.err || exit 1
  done
done
echo "rc=$?" >> $O/done.txt
