# Fixed-slot streaming kernel: software-counted waits (a_seq) vs tile-count waits (b_old), and a
# three-tile ring (c_seq_r3: read-only and records only, in place does not fit LDS); kbench passes.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for pass in 1 2; do
  for L in a_dyn b_static; do
    only="classify noswap nogroup,classify inplace nogroup,classify mac_out nogroup"
    [ $L = c_seq_r3 ] && only="classify noswap nogroup,classify mac_out nogroup"
    echo "== $L (pass $pass)"
    NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_$L.so timeout -k 10 300 python -u tools/kbench.py --only "$only" --no-multistream > gpurun_out/ab.log 2>&1
    rc=$?; grep median gpurun_out/ab.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab.log; exit $rc; }
  done
done
exit 0
