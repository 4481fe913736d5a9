# round 6, final tree: the driver's bench command once more on another box (the spread of the headline,
# the CPU baseline and the drop-in path from box to box), and smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_final5
mkdir -p $O
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
NBG_BENCH_FULL=$O/bench_full.json timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "rc=$?" >> $O/done.txt
