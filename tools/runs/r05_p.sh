# round 5: group_kernel ranks from a per-wave LDS peer-mask table (<= 128 bins) instead of the ballot
# multisplit: GPU suite, group launches alone (HEAD library vs tree, alternating), a bench without PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_p
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
for r in 0 1; do
  NBG_LIB_OVERRIDE=tools/ab/lib_head.so timeout -k 10 120 python3 tools/group_kbench.py --label head >> $O/kbench.txt 2>> $O/kbench.err || exit 1
  timeout -k 10 120 python3 tools/group_kbench.py --label peer >> $O/kbench.txt 2>> $O/kbench.err || exit 1
done &&
NBG_BENCH_FULL=$O/bench_full.json timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo "rc=$?" >> $O/done.txt
