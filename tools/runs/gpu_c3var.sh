# C3's MAC-handling variants (in place, 12-B records, read-only), tile-per-wave kernel, 3 streams;
# plus the records and read-only variants with NBG_STREAM_DESC on one stream.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
: > gpurun_out/c3var.txt
for v in in_place records read_only; do
  timeout -k 10 200 python -u tools/config_bench.py --config c3 --c3-variant $v > gpurun_out/c3v.json 2> gpurun_out/c3v.err || { tail -3 gpurun_out/c3v.err; exit 1; }
  cat gpurun_out/c3v.json | tee -a gpurun_out/c3var.txt
done
for v in records read_only; do
  echo "== stream-desc, 1 stream" | tee -a gpurun_out/c3var.txt
  timeout -k 10 200 python -u tools/config_bench.py --config c3 --c3-variant $v --streams 1 --stream-desc > gpurun_out/c3v.json 2> gpurun_out/c3v.err || { tail -3 gpurun_out/c3v.err; exit 1; }
  cat gpurun_out/c3v.json | tee -a gpurun_out/c3var.txt
  timeout -k 10 200 python -u tools/config_bench.py --config c3 --c3-variant $v --streams 1 > gpurun_out/c3v.json 2> gpurun_out/c3v.err || { tail -3 gpurun_out/c3v.err; exit 1; }
  cat gpurun_out/c3v.json | tee -a gpurun_out/c3var.txt
done
exit 0
