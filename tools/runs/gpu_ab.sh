# A/B of the libraries in tools/ab/ (single-stream and 4-stream C2 path variants)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
ONLY=${1:-"full path inplace,classify inplace nogroup,l2 inplace x4,classify only inplace x4"}
for pass in 1 2; do
  for L in tools/ab/lib_*.so; do
    echo "== $L (pass $pass)"
    NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 300 python -u tools/kbench.py --rounds 3 --streams 4 \
      --only "$ONLY" > gpurun_out/ab.log 2>&1
    rc=$?; grep median gpurun_out/ab.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab.log; exit $rc; }
  done
done
exit 0
