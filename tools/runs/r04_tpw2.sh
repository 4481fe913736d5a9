# round 4: C5 single launch with 1 / 2 / 4 tiles per wave (descriptors of all the wave's tiles loaded
# up front) now that the chain kernel has 56 VGPRs (8 waves per SIMD)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_tpw2
mkdir -p $O
timeout -k 10 300 python3 tools/imix_kbench.py --which c5,c3 --tpw 1,2,4 --rounds 2 --iters 40 > $O/kbench.txt 2>&1
echo "rc=$?" >> $O/done.txt
