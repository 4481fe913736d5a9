# round 4 final tree: kernel traces of the bench for profiles/ (launch shapes separated by
# tools/kshapes.py, ring completion stamps), then the --multi-only run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04_f2
mkdir -p $O/dump
NBG_BENCH_DUMP=$O/dump timeout -k 10 800 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --inline --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err &&
python3 tools/kshapes.py $O/trace $O/kshapes.csv > $O/kshapes.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/multi -o run --output-format csv -- python3 bench.py --inline --multi-only --steps 20 --warmup 5 > $O/multi_only.json 2> $O/multi_only.err &&
python3 tools/kshapes.py $O/multi $O/kshapes_multi.csv > $O/kshapes_multi.txt
echo "rc=$?" >> $O/done.txt
