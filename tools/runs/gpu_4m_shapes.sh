# read-only classify of one 4M-packet fixed-slot batch by kernel shape (kbench, no grouping):
# streaming (LDS-DMA), tile-per-wave with the L2-gathered LUT, tile-per-wave with the LDS LUT
cd "$GRAFT_REPO_ROOT" || exit 9
for pass in 1 2; do
  echo "== streaming (pass $pass)"
  timeout -k 10 300 python -u tools/kbench.py --n 4194304 --no-multistream --rounds 5 --only "classify noswap nogroup,classify inplace nogroup" 2>&1 | grep median
  echo "== tile-per-wave, L2 LUT (pass $pass)"
  NBG_STREAM=0 timeout -k 10 300 python -u tools/kbench.py --n 4194304 --no-multistream --rounds 5 --only "classify noswap nogroup,classify inplace nogroup" 2>&1 | grep median
  echo "== tile-per-wave, LDS LUT (pass $pass)"
  NBG_STREAM=0 timeout -k 10 300 python -u tools/kbench.py --n 4194304 --lut-lds --no-multistream --rounds 5 --only "classify noswap nogroup,classify inplace nogroup" 2>&1 | grep median
done
