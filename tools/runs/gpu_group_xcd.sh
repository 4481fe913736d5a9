# XCD-aware partition order in the group kernel (NBG_GROUP_XCD): C2 + C3 parity of the default
# build, then the per-batch C2 time (tools/overlap_probe.py) of base / xcd / no-perm-stores builds.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py > gpurun_out/xcd_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/xcd_pytest.log)"; [ $rc -ne 0 ] && exit $rc
for pass in 1 2 3; do
  for L in tools/ab/lib_*.so; do
    for cfg in in_place,1,3 read_only,1,3 records,1,3 in_place,1,1; do
      echo -n "$(basename $L) pass $pass: "
      NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 120 python tools/overlap_probe.py --steps 300 --warmup 30 --only $cfg 2> gpurun_out/gc.err
      rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/gc.err; exit $rc; }
    done
  done
done
exit 0
