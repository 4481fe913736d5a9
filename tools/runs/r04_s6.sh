# round 4: the bench (group burst 2, C4 shard multi-batch, C5 with the LDS LUT), membench with 256 MiB rewrites
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_s6
mkdir -p $O
hipcc -O3 --offload-arch=gfx950 -o tools/membench tools/membench.hip &&
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 180 ./tools/membench 32 > $O/membench32.txt 2>&1
echo "rc=$?" >> $O/done.txt
