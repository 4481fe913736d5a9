# round 6: 24-B header windows for direct host batches (frame bytes 14..37): the GPU suite, the drop-in
# sweep with its alternatives (48-B windows, ...); then C3's partition rows from the classify kernel's
# flush (NBG_HIST_KERNEL_BINS=2000) against hist_kernel, two alternating rounds of bench.py's variants
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_u
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 600 python3 tools/dropin_bench.py --extra > $O/dropin.json 2> $O/dropin.err || { echo "rc=$?" >> $O/done.txt; exit 1; }
F="--steps 5 --warmup 2 --no-ring --no-c4 --no-pmc --no-e2e --no-cpu-baseline"
for r in 0 1; do
  NBG_BENCH_FULL=$O/base_$r.json timeout -k 10 300 python3 bench.py $F > $O/base_$r.line 2> $O/base_$r.err &&
  NBG_HIST_KERNEL_BINS=2000 NBG_BENCH_FULL=$O/flush_$r.json timeout -k 10 300 python3 bench.py $F > $O/flush_$r.line 2> $O/flush_$r.err || break
done
echo "rc=$?" >> $O/done.txt
