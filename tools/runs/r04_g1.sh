# round 4: group kernel with 16-bit per-wave counters and packed sorted slots (40 KB of LDS at 1001
# bins instead of 64 KB) and classify blocks without an unused histogram: every GPU test, then the
# bench's C2 / C3 / C5 rates with the new library and with the previous one (lib_grpold), same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_g1
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
for lib in new old; do
  if [ $lib = old ]; then export NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_grpold.so; fi
  NBG_BENCH_IMIX_SWEEP=8x2 timeout -k 10 500 python3 bench.py --no-ring --no-pmc --no-cpu-baseline --no-c4 --steps 20 --warmup 5 > $O/bench_$lib.json 2> $O/bench_$lib.err || exit 1
done
echo "rc=$?" >> $O/done.txt
