# round 5: group-kernel A/B (committed kernel / prologue overlapped with the first chunk's ranks /
# wave-segment direct stores) through the whole bench, twice each; parity of the overlap build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_d
mkdir -p $O
NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_overlap.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_desc_multi.py tests/test_gpu_fuzz.py tests/test_gpu_ring.py > $O/tests_overlap.log 2>&1 &&
for r in 0 1; do for v in oldgroup overlap newgroup; do
  NBG_BENCH_FULL=$O/full_${v}_$r.json NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_$v.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit 1
done; done
echo "rc=$?" >> $O/done.txt
