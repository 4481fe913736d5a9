# PMC passes over kbench variants (single stream): SQ wave-state breakdown + TCP latency/stalls
cd "$GRAFT_REPO_ROOT" || exit 9
R0="$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_BUSY_CYCLES"
P2="TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES"
i=0
for V in "copy" "classify noswap" "classify inplace nogroup"; do
  for A in 0 1; do
    [ "$V" = "copy" ] && [ $A = 1 ] && continue
    for P in "$P1" "$P2"; do
      i=$((i+1))
      NBG_ABL=$A timeout -k 10 200 rocprofv3 --pmc $P --kernel-trace -d "$R0/gpurun_out/pmc$i" -o run --output-format csv -- python "$R0/tools/kbench.py" --no-multistream --rounds 1 --iters 10 --only "$V" > "$R0/gpurun_out/pmc$i.log" 2>&1
      rc=$?; echo "== $V ABL=$A pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$R0/gpurun_out/pmc$i.log"; exit $rc; }
      python "$R0/tools/pmcsum.py" "$R0/gpurun_out/pmc$i/run_counter_collection.csv" | grep -v "rocclr_fill"
    done
  done
done
exit 0
