# round 5, final tree (peer-mask group ranks, packed backend stores, XCD-aware group / compact / hist partitions): GPU suite, smoke, the
# driver's bench command (PMC traffic, end-to-end,
# CPU baseline), kernel traces of the bench and of --multi-only (csv, for tools/kshapes.py), then the two SQ
# PMC passes of tools/group_kbench.py
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_final5
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
NBG_BENCH_FULL=$O/bench_full.json timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 bench.py --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace_multi -o run -- python3 bench.py --multi-only --steps 50 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline > $O/bench_multi.json 2> $O/bench_multi.err &&
timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $O/g1 -o run -- python3 tools/group_kbench.py --iters 10 > $O/g1.txt 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d $O/g2 -o run -- python3 tools/group_kbench.py --iters 10 > $O/g2.txt 2>&1 &&
python3 tools/pmc_kernels.py $O/g1 > $O/pmc_g1.txt && python3 tools/pmc_kernels.py $O/g2 > $O/pmc_g2.txt
echo "rc=$?" >> $O/done.txt
