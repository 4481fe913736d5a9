# round 4: group kernel at <= 96 VGPRs (NBG_GROUP_WAVES 5; the bin-major scan re-reads its counters
# from LDS instead of holding 16 registers): parity, then the bench's C2 / C3 / C5 rates with the new
# library and HEAD's (lib_grpold), same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_gw
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_desc_multi.py tests/test_gpu_fuzz.py tests/test_gpu_ring.py > $O/tests.log 2>&1 &&
for lib in new old; do
  if [ $lib = old ]; then export NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_grpold.so; fi
  timeout -k 10 500 python3 bench.py --no-ring --no-c4 --no-pmc --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_$lib.json 2> $O/bench_$lib.err || exit 1
done
echo "rc=$?" >> $O/done.txt
