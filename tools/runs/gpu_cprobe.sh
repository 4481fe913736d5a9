# Per-wave launch timelines (tools/cprobe.py) for the classify variants, probe build.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_probe.so
for args in "--variant noswap" "--variant inplace" "--variant macout" "--variant noswap --lut-lds" "--variant inplace --lut-lds"; do
  for D in 0 1; do
    [ "$D" = 1 ] && [[ "$args" == *lut-lds* ]] && continue
    echo "######## NBG_DUAL=$D $args"
    NBG_DUAL=$D timeout -k 10 120 python -u tools/cprobe.py $args > gpurun_out/cprobe.log 2>&1
    rc=$?; cat gpurun_out/cprobe.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
