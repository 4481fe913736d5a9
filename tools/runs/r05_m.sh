# round 5: raw buffer loads (backends, partition rows) + packed row sums in group_kernel (tree) against
# 864a4d6 (base): GPU suite, probe, grouping launches alone, the whole bench twice each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_m
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 180 python3 tools/gprobe.py run > $O/gprobe.txt 2>&1 &&
for r in 0 1; do for v in tree base; do
  if [ $v = tree ]; then L=; else L=$PWD/tools/ab/lib_$v.so; fi
  NBG_LIB_OVERRIDE=$L timeout -k 10 120 python3 tools/group_kbench.py --label $v >> $O/gk.txt 2>> $O/gk.err || exit 1
done; done &&
for r in 0 1; do for v in tree base; do
  if [ $v = tree ]; then L=; else L=$PWD/tools/ab/lib_$v.so; fi
  NBG_BENCH_FULL=$O/full_${v}_$r.json NBG_LIB_OVERRIDE=$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit 1
done; done
echo "rc=$?" >> $O/done.txt
