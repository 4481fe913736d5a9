# round 4: what C5's routes longer than /24 (the dependent tbl_long gather) cost: 8 batches per launch
# with the full route set and with routes <= /24 only
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_c5long
mkdir -p $O
for p in 32 24 32 24; do
  timeout -k 10 200 python3 tools/imix_kbench.py --which c5 --multi 8 --iters 30 --max-plen $p >> $O/kbench.txt 2>&1 || exit 1
done
echo "rc=$?" >> $O/done.txt
