# round 4: descriptor multi path, classify and grouping launch times by batches per launch (1, 2, 4, 8),
# and C3 with the partition rows from the classify kernel (NBG_HIST_KERNEL_BINS=2000: no hist launch)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_dm2
mkdir -p $O
timeout -k 10 300 python3 tools/imix_kbench.py --which c3,c5 --multi 1,2,4,8 --rounds 2 --iters 30 > $O/kbench.txt 2>&1 &&
NBG_HIST_KERNEL_BINS=2000 timeout -k 10 200 python3 tools/imix_kbench.py --which c3 --multi 4,8 --rounds 2 --iters 30 > $O/kbench_histk.txt 2>&1
echo "rc=$?" >> $O/done.txt
