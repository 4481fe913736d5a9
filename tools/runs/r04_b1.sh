# round 4: the bench as the driver runs it, membench at 8 / 32 rotating buffers, membench PMC calibration
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_b1
O=gpurun_out/r04_b1
hipcc -O3 --offload-arch=gfx950 -o tools/membench tools/membench.hip &&
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 120 ./tools/membench 8 > $O/membench8.txt 2>&1 &&
timeout -k 10 180 ./tools/membench 32 > $O/membench32.txt 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/mb_fetch -o run --output-format csv -- ./tools/membench 32 10 > $O/mb_fetch.txt 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/mb_write -o run --output-format csv -- ./tools/membench 32 10 > $O/mb_write.txt 2>&1
echo "rc=$?" >> $O/done.txt
