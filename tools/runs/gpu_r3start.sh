# Session start: GPU suite + smoke, the default bench with rocprof stats, then the A/B libs in tools/ab.
cd "$GRAFT_REPO_ROOT" || exit 9
bash tools/gpu_suite.sh || exit $?
bash tools/runs/gpu_r2bench.sh || exit $?
bash tools/runs/gpu_ab_libs.sh --only "classify noswap nogroup,classify mac_out nogroup,classify inplace nogroup" --no-multistream --rounds 7
