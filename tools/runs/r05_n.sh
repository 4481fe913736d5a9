# round 5: PMC of the final grouping kernels (tools/group_kbench.py) and of the C3 / C5 classify at 8 per
# launch (tools/imix_kbench.py), two SQ passes each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_n
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"
timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $O/g1 -o run -- python3 tools/group_kbench.py --iters 10 > $O/g1.txt 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d $O/g2 -o run -- python3 tools/group_kbench.py --iters 10 > $O/g2.txt 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc $P1 --output-format csv -d $O/i1 -o run -- python3 tools/imix_kbench.py --which c3,c5 --multi 8 --iters 10 > $O/i1.txt 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc $P2 --output-format csv -d $O/i2 -o run -- python3 tools/imix_kbench.py --which c3,c5 --multi 8 --iters 10 > $O/i2.txt 2>&1 &&
python3 tools/pmc_kernels.py $O/g1 > $O/pmc_g1.txt && python3 tools/pmc_kernels.py $O/g2 > $O/pmc_g2.txt &&
python3 tools/pmc_kernels.py $O/i1 > $O/pmc_i1.txt && python3 tools/pmc_kernels.py $O/i2 > $O/pmc_i2.txt
echo "rc=$?" >> $O/done.txt
