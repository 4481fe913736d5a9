# round 5: phase timeline of group_kernel with the LDS peer-mask ranks (tools/gprobe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_q
mkdir -p $O
timeout -k 10 180 python3 tools/gprobe.py run > $O/gprobe.txt 2>&1
echo "rc=$?" >> $O/done.txt
