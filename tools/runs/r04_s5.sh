# round 4: C5 with the LDS-staged LUT; the grouped-ring tuning sweep; membench on the same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_s5
mkdir -p $O
hipcc -O3 --offload-arch=gfx950 -o tools/membench tools/membench.hip &&
timeout -k 10 200 python3 tools/imix_kbench.py --which c5,c3 --rounds 2 > $O/imix_default.txt 2>&1 &&
timeout -k 10 200 python3 tools/imix_kbench.py --which c5 --rounds 2 --lut-lds > $O/imix_lutlds.txt 2>&1 &&
NBG_BENCH_RING_GROUP_SWEEP=1 timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-imix --no-multi --no-pmc --no-cpu-baseline --no-c4 > $O/bench_gsweep.json 2> $O/bench_gsweep.err &&
timeout -k 10 180 ./tools/membench 32 > $O/membench32.txt 2>&1
echo "rc=$?" >> $O/done.txt
