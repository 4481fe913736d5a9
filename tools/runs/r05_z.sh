# round 5: packed backend stores in the streaming classify (lanes 0..7 store the wave's 128 B, as the ring does) vs one
# 2-B store per lane (tools/ab/lib_pack.so); parity of the C2 tests with it, then bench --multi-only alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_z
mkdir -p $O
NBG_LIB_OVERRIDE=tools/ab/lib_pack.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_multi.py > $O/tests_pack.log 2>&1 || exit 1
for r in 0 1 2; do
  for v in tree pack; do
    L=""; [ $v != tree ] && L=tools/ab/lib_$v.so
    NBG_LIB_OVERRIDE=$L NBG_BENCH_FULL=$O/full_${v}_$r.json timeout -k 10 200 python3 bench.py --multi-only --steps 50 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline >> $O/$v.jsonl 2>> $O/$v.err || exit 1
  done
done
echo "rc=$?" >> $O/done.txt
