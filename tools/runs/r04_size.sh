# round 4: classify time per 1M packets for C3 / C5 batches of 1M, 2M and 4M IMIX packets in one
# launch (is a multi-batch descriptor launch worth it?)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_size
mkdir -p $O
timeout -k 10 300 python3 tools/imix_kbench.py --which c3,c5 --n 1048576,2097152,4194304 --rounds 2 --iters 30 > $O/kbench.txt 2>&1
echo "rc=$?" >> $O/done.txt
