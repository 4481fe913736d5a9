# round 4: the chain with 2 tiles per wave, both tiles' windows in flight before the first tile's
# gathers (NBG_TPW=2): parity, then C5 one launch per batch and 8 per launch, against 1 tile per wave
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_pf2b
mkdir -p $O
NBG_TPW=2 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lpm.py tests/test_gpu_desc_multi.py tests/test_gpu_fuzz.py -k "chain or lpm or desc" > $O/tests.log 2>&1 &&
for r in 1 2; do
  timeout -k 10 200 python3 tools/imix_kbench.py --which c5 --tpw 1,2 --iters 40 >> $O/kbench_single.txt 2>&1 &&
  timeout -k 10 200 python3 tools/imix_kbench.py --which c5 --multi 8 --iters 30 >> $O/kbench_multi_tpw1.txt 2>&1 &&
  NBG_TPW=2 timeout -k 10 200 python3 tools/imix_kbench.py --which c5 --multi 8 --iters 30 >> $O/kbench_multi_tpw2.txt 2>&1 || exit 1
done
echo "rc=$?" >> $O/done.txt
