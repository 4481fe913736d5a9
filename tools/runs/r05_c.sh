# round 5: new group kernel (wave-segment ranks, direct perm stores): whole GPU suite, smoke, C3
# multi-launch classify / grouping times with the partial write-back A/B, membench (32-B sector
# rewrites), the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_c
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 200 python3 tools/imix_kbench.py --which c3,c5 --multi 8 --wb-partial 0,1 --rounds 2 --iters 30 > $O/imix_multi.json 2> $O/imix_multi.err &&
timeout -k 10 300 ./tools/membench 32 50 > $O/membench32.txt 2>&1 &&
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
cp gpurun_out/bench_full_latest.json $O/bench_full.json
echo "rc=$?" >> $O/done.txt
