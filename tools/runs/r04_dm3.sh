# round 4: C3 / C5 multi-batch descriptor path, whole-job rate by batches per launch x streams
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_dm3
mkdir -p $O
NBG_BENCH_IMIX_SWEEP=2x3,4x2,4x3,8x2 timeout -k 10 600 python3 bench.py --no-ring --no-pmc --no-cpu-baseline --no-c4 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "rc=$?" >> $O/done.txt
