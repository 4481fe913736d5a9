# round 4: C5 with the LDS-staged LUT, gate resolved one tile later (NBG_GATHER_LAG, in-tree) vs
# resolved in the same tile (lib_nolag): parity, then classify time on one stream
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_lag
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lpm.py tests/test_gpu_fuzz.py -k "chain or lpm" > $O/tests.log 2>&1 &&
for round in 1 2; do
  timeout -k 10 120 python3 tools/imix_kbench.py --which c5 --lut-lds >> $O/kbench.txt 2>&1 &&
  NBG_LIB_OVERRIDE=$PWD/tools/ab/lib_nolag.so timeout -k 10 120 python3 tools/imix_kbench.py --which c5 --lut-lds >> $O/kbench.txt 2>&1 &&
  timeout -k 10 120 python3 tools/imix_kbench.py --which c5 >> $O/kbench.txt 2>&1 || exit 1
done
echo "rc=$?" >> $O/done.txt
