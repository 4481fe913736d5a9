# A/B of tools/ab/lib_*.so: single-stream classify variants and the 3-stream full path (kbench), two passes.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for pass in 1 2; do
  for L in tools/ab/lib_*.so; do
    echo "== $L (pass $pass)"
    NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 300 python -u tools/kbench.py --streams 3 --rounds 5 \
      --only "classify noswap nogroup,classify mac_out nogroup,classify inplace nogroup,full path l2 inplace x3,full path l2 mac_out x3,classify only inplace x3,full path l2 noswap x3" > gpurun_out/ab.log 2>&1
    rc=$?; grep median gpurun_out/ab.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab.log; exit $rc; }
  done
done
exit 0
