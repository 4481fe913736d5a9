# round 4: the 4 x 1M fixed-slot multi launch without the per-unit partition-row flush
# (NBG_MULTI_HIST_KERNEL=1: one hist_kernel launch beside the group launch): parity, then C2 in place,
# alternating, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_mh
mkdir -p $O
NBG_MULTI_HIST_KERNEL=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_multi.py tests/test_gpu_desc_multi.py > $O/tests.log 2>&1 &&
for r in 1 2; do
  timeout -k 10 200 python3 tools/c2_multik.py --k 4 --rounds 1 >> $O/c2_base.txt 2>&1 &&
  NBG_MULTI_HIST_KERNEL=1 timeout -k 10 200 python3 tools/c2_multik.py --k 4 --rounds 1 >> $O/c2_histk.txt 2>&1 || exit 1
done
echo "rc=$?" >> $O/done.txt
