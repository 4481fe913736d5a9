# round 4: descriptor multi-batch path (C3 / C5, several IMIX batches per launch): parity, then the
# bench's IMIX variants (single-batch launches on 3 streams vs 4 batches per launch on 2 streams)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_dm1
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_desc_multi.py tests/test_gpu_multi.py tests/test_gpu_lpm.py tests/test_gpu_parity.py > $O/tests.log 2>&1 &&
timeout -k 10 400 python3 bench.py --no-ring --no-pmc --no-cpu-baseline --no-c4 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "rc=$?" >> $O/done.txt
