# round 4: C2 in place with 4 vs 8 batches per multi-batch launch (2 streams, 16 distinct inputs)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_k8
mkdir -p $O
timeout -k 10 300 python3 tools/c2_multik.py --k 4,8 --rounds 2 > $O/c2_multik.txt 2>&1
echo "rc=$?" >> $O/done.txt
