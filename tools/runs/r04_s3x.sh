# round 4: C3 / C5 at 8 batches per launch on 3 streams against 2 (same run)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_s3x
mkdir -p $O
NBG_BENCH_IMIX_SWEEP=8x3,8x2,8x3 timeout -k 10 700 python3 bench.py --no-ring --no-c4 --no-pmc --no-cpu-baseline --no-multi --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "rc=$?" >> $O/done.txt
