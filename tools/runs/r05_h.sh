# round 5: grouping launches alone (tools/group_kbench.py): the tree, the round-4 group kernel, and
# the tree without the direct prefix's row loads (ablation, timing only); then a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_h
mkdir -p $O
for r in 0 1; do for v in tree oldgroup norows; do
  if [ $v = tree ]; then L=; else L=$PWD/tools/ab/lib_$v.so; fi
  NBG_LIB_OVERRIDE=$L timeout -k 10 120 python3 tools/group_kbench.py --label $v >> $O/gk.txt 2>> $O/gk.err || exit 1
done; done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/group_kbench.py --label tree_prof >> $O/gk.txt 2>> $O/gk.err
echo "rc=$?" >> $O/done.txt
