# Streaming classify vs the tile-per-wave kernel (NBG_STREAM=0/1) in one GPU call: GPU parity with
# the default (streaming), then kbench passes interleaved across the two.  Extra args go to kbench.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for S in 0 1; do
    echo "== NBG_STREAM=$S (pass $pass)"
    NBG_STREAM=$S timeout -k 10 300 python -u tools/kbench.py "$@" > gpurun_out/ab.log 2>&1
    rc=$?; grep median gpurun_out/ab.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab.log; exit $rc; }
  done
done
