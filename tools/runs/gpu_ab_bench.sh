# A/B of tools/ab/lib_*.so through bench.py itself (classify with grouping deferred, per variant,
# plus the 3-stream value), two interleaved passes; C2 parity of the default build first.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "c2 or multi_chunk or no_swap or mac_out or repeat or many_backends_multi" > gpurun_out/ab_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/ab_pytest.log; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for L in tools/ab/lib_*.so; do
    echo "== $L (pass $pass)"
    NBG_LIB_OVERRIDE=$PWD/$L timeout -k 10 300 python bench.py --inline --no-pmc --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err
    rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab_bench.err; exit $rc; }
    python - <<'PY'
import json
d = json.load(open("gpurun_out/ab_bench.json"))
r = d["roofline"]; v = d.get("variants", {})
print(f"  value {d['value']:.0f} Mpps | in_place {r['avg_launch_us']} us (group {r['group_kernel_avg_us']})"
      + "".join(f" | {k} {x['avg_launch_us']} us value {x['value']:.0f}" for k, x in v.items()))
PY
  done
done
exit 0
