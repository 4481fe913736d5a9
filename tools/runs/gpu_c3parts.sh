# C3 grouping with partitions of 1, 2, 4 chunks (NBG_PART_CHUNKS_WIDE), in place and read-only,
# after the many-backend parity tests with 2-chunk partitions.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
NBG_PART_CHUNKS_WIDE=2 timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "c3_full or many_backends or imix_descriptors" > gpurun_out/parts_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/parts_pytest.log; [ $rc -ne 0 ] && exit $rc
for v in in_place read_only; do
  for c in 1 2 4; do
    echo "== $v chunks=$c"
    NBG_PART_CHUNKS_WIDE=$c timeout -k 10 200 python -u tools/config_bench.py --config c3 --c3-variant $v > gpurun_out/cp.json 2> gpurun_out/cp.err || { tail -3 gpurun_out/cp.err; exit 1; }
    cat gpurun_out/cp.json
  done
done
exit 0
