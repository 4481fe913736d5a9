# round 6: why the 20-step headline runs ~5 % under its 50-step steady state.  The same bench line
# (headline + steady only) with 5, 30 and 100 warmup steps, and a kernel trace of the 5-warmup run
# (the headline's per-call durations and gaps, first calls against last)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_k
mkdir -p $O
F="--no-variants --no-pmc --no-e2e --no-cpu-baseline --no-c4"
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 $F > $O/w5.json 2> $O/w5.err &&
timeout -k 10 200 python3 bench.py --steps 20 --warmup 30 $F > $O/w30.json 2> $O/w30.err &&
timeout -k 10 200 python3 bench.py --steps 20 --warmup 100 $F > $O/w100.json 2> $O/w100.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ktrace -o run -- python3 bench.py --steps 20 --warmup 5 $F > $O/prof.json 2> $O/prof.err
echo "rc=$?" >> $O/done.txt
# the multi launch with and without the classify kernel's per-unit histogram (verdict item 5)
timeout -k 10 200 python3 tools/c2_multik.py --k 4,8 --nohist > $O/multik.json 2> $O/multik.err
echo "rc2=$?" >> $O/done.txt
