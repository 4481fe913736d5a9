# round 5: PMC of the grouping kernels (tools/group_kbench.py; two SQ passes, counters per kernel by
# tools/pmc_kernels.py): where group_kernel's time goes (VALU / LDS / waits)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_k
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/p1 -o run -- python3 tools/group_kbench.py --iters 10 > $O/p1.txt 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM --output-format csv -d $O/p2 -o run -- python3 tools/group_kbench.py --iters 10 > $O/p2.txt 2>&1 &&
python3 tools/pmc_kernels.py $O/p1 > $O/pmc1.txt && python3 tools/pmc_kernels.py $O/p2 > $O/pmc2.txt
echo "rc=$?" >> $O/done.txt
