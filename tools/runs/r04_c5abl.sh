# round 4: where C5's classify time goes (tbl24 gather, LUT gather, gate stores), descriptor prefetch
# with 2-4 tiles per wave (NBG_TPW) and the next tile's windows in flight (lib_pf2), A/B builds in one call
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_c5abl.txt
: > $O
for round in 1 2; do
  for lib in cur pf2; do
    [ -f tools/ab/lib_$lib.so ] || continue
    NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_$lib.so timeout -k 10 200 python3 tools/imix_kbench.py --which c5,c3 --tpw 1,2,4 >> $O 2>&1 || { echo "FAIL $lib" >> $O; exit 1; }
  done
  for lib in base c5abl1 c5abl2 c5abl4 c5abl7; do
    NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_$lib.so timeout -k 10 120 python3 tools/imix_kbench.py --which c5 >> $O 2>&1 || { echo "FAIL $lib" >> $O; exit 1; }
  done
done
timeout -k 10 120 python3 tools/imix_kbench.py --which c5,c3 --stream-desc >> $O 2>&1
echo "rc=$?" >> $O
