# round 5: hist_kernel in the group kernel's XCD-aware partition order (the group block of partition c then
# re-reads the backends hist_kernel read on the same XCD) vs the previous commit (tools/ab/lib_head3.so);
# grouping tests, group launches alone, the bench without ring / C4 / PMC, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_ac
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_desc_multi.py tests/test_gpu_ring.py tests/test_gpu_group_compact.py > $O/tests.log 2>&1 || exit 1
for r in 0 1; do
  for v in head3 tree; do
    L=""; [ $v != tree ] && L=tools/ab/lib_$v.so
    NBG_LIB_OVERRIDE=$L timeout -k 10 120 python3 tools/group_kbench.py --label $v >> $O/kbench.txt 2>> $O/kbench.err || exit 1
  done
done
for r in 0 1; do
  for v in head3 tree; do
    L=""; [ $v != tree ] && L=tools/ab/lib_$v.so
    NBG_LIB_OVERRIDE=$L NBG_BENCH_FULL=$O/full_${v}_$r.json timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline --no-c4 > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit 1
  done
done
echo "rc=$?" >> $O/done.txt
