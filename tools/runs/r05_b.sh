# round 5: the whole GPU suite on the cleaned library (probe builds removed, ring lifecycle), smoke,
# then the C3 partial write-back A/B (classify time; WRITE_SIZE / FETCH_SIZE of the multi launch)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_b
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 200 python3 tools/imix_kbench.py --which c3 --multi 8 --wb-partial 0,1 --rounds 2 --iters 30 > $O/c3_wbp.json 2> $O/c3_wbp.err &&
timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_w -o run --output-format csv -- python3 tools/imix_kbench.py --which c3 --multi 8 --wb-partial 0,1 --iters 10 > $O/pmc_w.out 2>&1 &&
timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_f -o run --output-format csv -- python3 tools/imix_kbench.py --which c3 --multi 8 --wb-partial 0,1 --iters 10 > $O/pmc_f.out 2>&1
echo "rc=$?" >> $O/done.txt
