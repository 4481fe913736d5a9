# Batch-size scaling of the classify kernel (per-launch overhead vs streaming rate) and the
# NBG_ABL ablations, one process per setting, same box.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
V="classify noswap nogroup,classify inplace nogroup,classify mac_out nogroup,copy"
for N in 1048576 4194304; do
  echo "== n=$N"
  timeout -k 10 300 python -u tools/kbench.py --n $N --rounds 3 --no-multistream --only "$V" > gpurun_out/scale.log 2>&1
  rc=$?; grep median gpurun_out/scale.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/scale.log; exit $rc; }
done
for A in 1 3 4; do
  echo "== ABL=$A n=1M"
  NBG_ABL=$A timeout -k 10 300 python -u tools/kbench.py --rounds 3 --no-multistream --only "classify noswap nogroup" > gpurun_out/scale.log 2>&1
  rc=$?; grep median gpurun_out/scale.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/scale.log; exit $rc; }
done
timeout -k 10 120 ./tools/membench > gpurun_out/membench.log 2>&1; rc=$?; cat gpurun_out/membench.log; exit $rc
