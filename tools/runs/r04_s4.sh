# round 4: C5 / C3 A/B (ablations, tiles per wave, window prefetch), then the full bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_s4
mkdir -p $O
timeout -k 10 600 bash tools/runs/r04_c5abl.sh &&
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "rc=$?" >> $O/done.txt
