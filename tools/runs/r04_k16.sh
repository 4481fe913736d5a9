# round 4: up to 16 batches per multi-batch launch (NBG_MAX_MULTI 16): parity, then C3 / C5 at 16
# batches per launch against 8 (same run)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_k16
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_desc_multi.py tests/test_gpu_multi.py tests/test_gpu_ring.py > $O/tests.log 2>&1 &&
NBG_BENCH_IMIX_SWEEP=16x2,8x2 timeout -k 10 600 python3 bench.py --no-ring --no-c4 --no-pmc --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "rc=$?" >> $O/done.txt
