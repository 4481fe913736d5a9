# Group-kernel chunk / partition sizes (tools/ab builds): C2 parity per build, then the per-batch
# time of the C2 path at 3 and 1 streams (tools/overlap_probe.py), two interleaved passes.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for L in tools/ab/lib_*.so; do
  NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "c2 or multi_chunk or no_swap or many_backends" > gpurun_out/chunk_pytest.log 2>&1
  rc=$?; echo "$(basename $L) parity rc=$rc $(tail -1 gpurun_out/chunk_pytest.log)"; [ $rc -ne 0 ] && exit $rc
done
for pass in 1 2; do
  for L in tools/ab/lib_*.so; do
    for cfg in in_place,1,3 read_only,1,3 records,1,3 in_place,1,1 read_only,1,1; do
      echo -n "$(basename $L) pass $pass: "
      NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 120 python tools/overlap_probe.py --steps 300 --warmup 30 --only $cfg 2> gpurun_out/gc.err
      rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/gc.err; exit $rc; }
    done
  done
done
exit 0
