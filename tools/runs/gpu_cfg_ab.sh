# Config A/B in one call: C3 histograms in classify (NBG_HIST_KERNEL_BINS=2000) vs hist_kernel, and
# C5 with the LDS-staged LUT (--lut-lds) vs the L2 gather; two passes.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
: > gpurun_out/cfg_ab.txt
run() {  # label, env, args
  echo "== $1" | tee -a gpurun_out/cfg_ab.txt
  env $2 timeout -k 10 200 python -u tools/config_bench.py $3 > gpurun_out/cfg.json 2> gpurun_out/cfg.err || { tail -3 gpurun_out/cfg.err; exit 1; }
  cat gpurun_out/cfg.json | tee -a gpurun_out/cfg_ab.txt
}
for pass in 1 2; do
  run "c3 hist_kernel" "NBG_HIST_KERNEL_BINS=257" "--config c3"
  run "c3 hist in classify" "NBG_HIST_KERNEL_BINS=2000" "--config c3"
  run "c5 L2 LUT" "NBG_X=0" "--config c5"
  run "c5 LDS LUT" "NBG_X=0" "--config c5 --lut-lds"
done
exit 0
