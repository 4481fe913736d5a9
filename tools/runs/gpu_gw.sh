# group-kernel register budget (NBG_GROUP_WAVES builds in tools/ab/): 4-stream full path, C2 and C3
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for pass in 1 2 3; do
  for L in tools/ab/lib_*.so; do
    echo "== $L (pass $pass)"
    NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 300 python -u tools/kbench.py --rounds 3 --streams 4 \
      --only "full path inplace,x4 streams" > gpurun_out/ab.log 2>&1
    rc=$?; grep median gpurun_out/ab.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab.log; exit $rc; }
  done
done
exit 0
