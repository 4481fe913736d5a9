# round 5: XCD-aware partition order in group_kernel (tools/ab/lib_xcd.so: XCD x takes a contiguous eighth of
# the partitions, so the pieces of a perm line written by neighbouring partitions meet in one L2) vs the tree;
# parity of the grouping tests with it, then group launches alone and the bench's C3 / C5 / C2 multi paths
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_aa
mkdir -p $O
NBG_LIB_OVERRIDE=tools/ab/lib_xcd.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_desc_multi.py > $O/tests_xcd.log 2>&1 || exit 1
for r in 0 1; do
  for v in tree xcd; do
    L=""; [ $v != tree ] && L=tools/ab/lib_$v.so
    NBG_LIB_OVERRIDE=$L timeout -k 10 120 python3 tools/group_kbench.py --label $v >> $O/kbench.txt 2>> $O/kbench.err || exit 1
  done
done
for r in 0 1; do
  for v in tree xcd; do
    L=""; [ $v != tree ] && L=tools/ab/lib_$v.so
    NBG_LIB_OVERRIDE=$L NBG_BENCH_FULL=$O/full_${v}_$r.json timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline --no-ring --no-c4 > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit 1
  done
done
echo "rc=$?" >> $O/done.txt
