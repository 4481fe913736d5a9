# C3 decomposition: IMIX layout with different LUT size / width / modulus
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for cfg in "65 65537" "1000 65537" "65 655373" "1000 655373"; do
  set -- $cfg
  echo "== nb=$1 m=$2"
  timeout -k 10 300 python tools/kbench.py --mode 1 --nb $1 --m $2 --rounds 3 --iters 20 --no-multistream --only "classify noswap,classify mac_out,classify inplace nogroup,counts" > gpurun_out/c3ab.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/c3ab.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
