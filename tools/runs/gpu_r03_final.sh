#!/bin/bash
# Round 3 final measurement set: the whole -m gpu suite + smoke, the default bench line, and a
# rocprofv3 kernel-trace/stats profile of the bench's single-rank run.
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail -20 gpurun_out/final_bench.err; exit 1; }
cut -c1-400 gpurun_out/final_bench.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R0/gpurun_out/final_prof" -o run --output-format csv -- python3 "$R0/bench.py" --inline --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > "$R0/gpurun_out/final_prof_bench.json" 2> "$R0/gpurun_out/final_prof.err" || { echo "profile failed"; tail -20 "$R0/gpurun_out/final_prof.err"; exit 1; }
cd "$R0" && find gpurun_out/final_prof -name "*kernel_stats.csv" | head -3
echo done
