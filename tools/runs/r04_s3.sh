# round 4: the bench's C4 block alone (the last run went silent there), then the full bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_s3
mkdir -p $O
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-variants --no-pmc --no-cpu-baseline > $O/c4only.json 2> $O/c4only.err &&
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "rc=$?" >> $O/done.txt
