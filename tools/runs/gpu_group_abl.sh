# Group-kernel ablations (NBG_GABL builds, wrong perm by design): the 3-stream C2 per-batch time
# (tools/overlap_probe.py), two interleaved passes.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for pass in 1 2; do
  for L in tools/ab/lib_*.so; do
    for cfg in in_place,1,3 read_only,1,3; do
      echo -n "$(basename $L) pass $pass: "
      NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 120 python tools/overlap_probe.py --steps 300 --warmup 30 --only $cfg 2> gpurun_out/gc.err
      rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/gc.err; exit $rc; }
    done
  done
done
exit 0
