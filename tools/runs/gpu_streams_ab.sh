# bench value (C2 in place + grouping) by stream count, three interleaved passes
cd "$GRAFT_REPO_ROOT" || exit 9
for pass in 1 2 3; do
  for S in 2 3 4; do
    timeout -k 10 200 python bench.py --inline --no-pmc --no-cpu-baseline --no-variants --streams $S > gpurun_out/s.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/s.json')); print('pass $pass streams $S', d['value'], d['ms_per_step'])"
  done
done
