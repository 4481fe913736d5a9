# round 4 session 2: full GPU suite (descriptor prefetch, chunk-3 skip, repeated ring inputs), the bench
# with the ring producers' in-flight cap, and the C5 ablation / tiles-per-wave A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04_s2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 500 bash tools/runs/r04_c5abl.sh
echo "rc=$?" >> $O/done.txt
