cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
: > gpurun_out/zc_all.txt
for a in "--streams 1" "--streams 2" "--streams 3" "--thp --streams 2" "--room 64 --streams 2"; do
  timeout -k 10 200 python -u tools/zerocopy_probe.py $a > gpurun_out/zc.json 2> gpurun_out/zc.err
  rc=$?; echo "== $a rc=$rc" | tee -a gpurun_out/zc_all.txt; cat gpurun_out/zc.json | tee -a gpurun_out/zc_all.txt
  [ $rc -ne 0 ] && { tail -5 gpurun_out/zc.err; exit $rc; }
done
exit 0
