# C3: partition histograms in the classify kernel's flush (NBG_HIST_KERNEL_BINS=2000) against
# hist_kernel (default for > 256 bins), config_bench C3, two passes.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for pass in 1 2; do
  for B in 257 2000; do
    echo "== NBG_HIST_KERNEL_BINS=$B (pass $pass)"
    NBG_HIST_KERNEL_BINS=$B timeout -k 10 200 python -u tools/config_bench.py --config c3 > gpurun_out/c3h.json 2> gpurun_out/c3h.err || { tail -3 gpurun_out/c3h.err; exit 1; }
    cat gpurun_out/c3h.json
  done
done
exit 0
