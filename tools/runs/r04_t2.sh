# round 4: the descriptor multi-batch tests (incl. beside a running ring); then C5 / C3 single launch
# with 1 / 2 / 4 tiles per wave now that the chain kernel has 56 VGPRs (8 waves per SIMD)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_t2
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_desc_multi.py > $O/tests.log 2>&1 &&
timeout -k 10 300 python3 tools/imix_kbench.py --which c5,c3 --tpw 1,2,4 --rounds 2 --iters 40 > $O/kbench_tpw.txt 2>&1
echo "rc=$?" >> $O/done.txt
