# 48-B vs 64-B LDS rows for read-only / records (tools/ab libs): kbench one stream + multi, two passes
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for pass in 1 2; do
  for L in tools/ab/lib_*.so; do
    echo "== $L (pass $pass)"
    NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 300 python -u tools/kbench.py --no-multistream --rounds 5 --only "classify noswap nogroup,classify mac_out nogroup,multi4 noswap,multi4 mac_out" > gpurun_out/ab.log 2>&1
    rc=$?; grep median gpurun_out/ab.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab.log; exit $rc; }
    NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 200 python tools/multi_probe.py 2>/dev/null | grep "read-only, hist"
  done
done
