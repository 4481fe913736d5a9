# Descriptor streaming kernel ablations (tools/ab/lib_*.so built with NBG_DABL): classify alone,
# C5 and C3, one stream; plus the tile-per-wave kernel (NBG_STREAM=0) of lib_base.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for L in base nogather nopkt none; do
  echo "== $L"
  NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_$L.so timeout -k 10 300 python -u tools/config_bench.py --config c5,c3 --streams 1 > gpurun_out/abl.log 2>&1
  rc=$?; grep -o '"config": "c.", "mpps": [0-9.]*\|"classify_us": [0-9.]*' gpurun_out/abl.log | paste - - - -; [ $rc -ne 0 ] && { tail -5 gpurun_out/abl.log; exit $rc; }
done
echo "== tile-per-wave"
NBG_STREAM=0 NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_base.so timeout -k 10 300 python -u tools/config_bench.py --config c5,c3 --streams 1 > gpurun_out/abl.log 2>&1
grep -o '"config": "c.", "mpps": [0-9.]*\|"classify_us": [0-9.]*' gpurun_out/abl.log | paste - - - -
exit 0
