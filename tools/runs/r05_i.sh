# round 5: unrolled perm stores + paired 10-bit chunk scan (tree) against the first rework (v2 =
# bfa9bec) and a constant-rows ablation of the tree (timing only); GPU suite and probe of the tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_i
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 180 python3 tools/gprobe.py run > $O/gprobe.txt 2>&1 &&
for r in 0 1; do for v in tree v2 constrows; do
  if [ $v = tree ]; then L=; else L=$PWD/tools/ab/lib_$v.so; fi
  NBG_LIB_OVERRIDE=$L timeout -k 10 120 python3 tools/group_kbench.py --label $v >> $O/gk.txt 2>> $O/gk.err || exit 1
done; done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/group_kbench.py --label tree_prof >> $O/gk.txt 2>> $O/gk.err
echo "rc=$?" >> $O/done.txt
