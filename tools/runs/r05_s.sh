# round 5: the LDS peer-mask ranks for up to 1023 bins (7-bit-keyed table + 3 ballots) vs up to 128 only:
# GPU suite, group launches alone (alternating), a bench without PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_s
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
for r in 0 1; do
  NBG_LIB_OVERRIDE=tools/ab/lib_peer7.so timeout -k 10 120 python3 tools/group_kbench.py --label peer7 >> $O/kbench.txt 2>> $O/kbench.err || exit 1
  timeout -k 10 120 python3 tools/group_kbench.py --label peer10 >> $O/kbench.txt 2>> $O/kbench.err || exit 1
done &&
for v in peer7 peer10 peer7 peer10; do
  L=""; [ $v = peer7 ] && L=tools/ab/lib_peer7.so
  NBG_LIB_OVERRIDE=$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline --no-ring --no-c4 >> $O/bench_$v.jsonl 2>> $O/bench_$v.err || exit 1
done
echo "rc=$?" >> $O/done.txt
