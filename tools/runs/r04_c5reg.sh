# round 4: the chain kernel with the MAC-swap write-back compiled out (the tile's registers die after
# the transpose: 56 VGPRs instead of 68, 8 waves per SIMD instead of 7) against HEAD (lib_c5old):
# parity, then C5 classify at 8 and 1 batches per launch, alternating, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_c5reg
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lpm.py tests/test_gpu_desc_multi.py tests/test_gpu_fuzz.py -k "chain or lpm or desc" > $O/tests.log 2>&1 &&
for r in 1 2; do
  timeout -k 10 200 python3 tools/imix_kbench.py --which c5 --multi 1,8 --iters 30 >> $O/kbench_new.txt 2>&1 &&
  NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_c5old.so timeout -k 10 200 python3 tools/imix_kbench.py --which c5 --multi 1,8 --iters 30 >> $O/kbench_old.txt 2>&1 || exit 1
done
echo "rc=$?" >> $O/done.txt
