# PMC: LDS and VMEM issue detail for classify noswap (ABL 0/1/2) and copy
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp
P3="SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAVE_CYCLES"
P4="SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU"
i=20
for V in "copy" "classify noswap"; do
  for A in 0 1; do
    [ "$V" = "copy" ] && [ $A = 1 ] && continue
    for P in "$P3" "$P4"; do
      i=$((i+1))
      NBG_ABL=$A timeout -k 10 200 rocprofv3 --pmc $P --kernel-trace -d "$R0/gpurun_out/pmc$i" -o run --output-format csv -- python "$R0/tools/kbench.py" --no-multistream --rounds 1 --iters 10 --only "$V" > "$R0/gpurun_out/pmc$i.log" 2>&1
      rc=$?; echo "== $V ABL=$A pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$R0/gpurun_out/pmc$i.log"; exit $rc; }
      python "$R0/tools/pmcsum.py" "$R0/gpurun_out/pmc$i/run_counter_collection.csv" | grep -v "rocclr_fill" | grep -A9 "classify\|copyBuffer"
    done
  done
done
exit 0
