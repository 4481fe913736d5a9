# C3/C5 (config_bench) per tools/ab/lib_*.so: default kernels at 3 and 1 streams, the descriptor
# streaming kernel at 1 stream; two interleaved passes.  Prints mpps, us/batch, classify us.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for pass in 1 2; do
  for L in tools/ab/lib_*.so; do
    for args in "--streams 3" "--streams 1" "--streams 1 --stream-desc"; do
      NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 200 python tools/config_bench.py --steps 100 --warmup 10 $args > gpurun_out/cfg.json 2> gpurun_out/cfg.err
      rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/cfg.err; exit $rc; }
      python -c "
import json,sys
for l in open('gpurun_out/cfg.json'):
    d=json.loads(l); print(sys.argv[1], sys.argv[2], '|', d['config'], 'Mpps', d['mpps'], 'us/batch', d['us_per_batch'], 'classify_us', d['classify_us'])" "$(basename $L .so) p$pass" "$args"
    done
  done
done
