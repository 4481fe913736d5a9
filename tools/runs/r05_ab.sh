# round 5: XCD-aware partition order in the compact group kernel (group_direct_kernel, taken beside a running
# ring for many bins; NBG_GROUP_COMPACT=1 forces it here) vs the previous commit's library (tools/ab/lib_head2.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_ab
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_group_compact.py tests/test_gpu_ring.py > $O/tests.log 2>&1 || exit 1
for r in 0 1; do
  for v in head2 tree; do
    L=""; [ $v != tree ] && L=tools/ab/lib_$v.so
    NBG_GROUP_COMPACT=1 NBG_LIB_OVERRIDE=$L timeout -k 10 120 python3 tools/group_kbench.py --label compact_$v >> $O/kbench.txt 2>> $O/kbench.err || exit 1
  done
done
echo "rc=$?" >> $O/done.txt
