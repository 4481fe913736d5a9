# A/B of the libraries in tools/ab/ on the bench's own step (default 3 streams), in place and records
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for pass in 1 2; do
  for L in tools/ab/lib_*.so; do
    for M in "" "--mac-record"; do
      NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 200 python bench.py --no-cpu-baseline $M > gpurun_out/bab.json 2> gpurun_out/bab.err
      rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/bab.err; exit $rc; }
      python -c "import json;d=json.load(open('gpurun_out/bab.json'));print('$L', '${M:-inplace}', d['value'], d['ms_per_step'])"
    done
  done
done
exit 0
