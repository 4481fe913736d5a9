# round 4: C5 at 8 batches per launch with the partition rows from the classify kernel (default) or
# from hist_kernel on the grouping stream (NBG_HIST_KERNEL_BINS=1); then the bench with its PMC passes
# (now including the descriptor multi-batch launches)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_h1
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python3 tools/imix_kbench.py --which c5 --multi 8 --iters 30 >> $O/kbench_default.txt 2>&1 &&
  NBG_HIST_KERNEL_BINS=1 timeout -k 10 200 python3 tools/imix_kbench.py --which c5 --multi 8 --iters 30 >> $O/kbench_histk.txt 2>&1 || exit 1
done
timeout -k 10 600 python3 bench.py --no-ring --no-c4 --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "rc=$?" >> $O/done.txt
