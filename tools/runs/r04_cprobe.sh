# round 4: per-wave timelines of one classify launch (probe build): C5's chain on a 1M IMIX batch,
# and C2's tile-per-wave kernel read only for comparison
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_cprobe
mkdir -p $O
export NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_probe.so
for v in c5 noswap; do
  timeout -k 10 120 python3 -u tools/cprobe.py --variant $v > $O/cprobe_$v.txt 2>&1 || exit 1
done
echo "rc=$?" >> $O/done.txt
