# round 6: the small kernel's perm staged in LDS and stored in order (16 B per lane), backend[] stored after every round's gathers
# instead of scattered 4-B stores: the GPU tests of the small kernel and the host paths, the server timeline again (probe
# build of this tree), and an A/B of this tree against HEAD's library (tools/ab/base) in the drop-in
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_y
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_host_ring.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_zerocopy.py tests/test_gpu_fuzz.py > $O/tests.log 2>&1 &&
python3 tools/dropin_bench.py --write-pcap $O/c1.pcap &&
for p in 1 16; do
  LD_LIBRARY_PATH=$PWD/tools/ab/hrprobe NBG_PROBE_OUT=$O/p$p.bin timeout -k 10 120 netbricks_amd/host/nb_maglev --rx $O/c1.pcap --backends 65 --batch 992 --loop 3000000 --pipelines $p --host-ring 64 > $O/p$p.json 2> $O/p$p.err || break
  python3 tools/hrprobe_stats.py $O/p$p.bin > $O/p$p.stats || break
done &&
timeout -k 10 600 python3 tools/dropin_bench.py --ab-lib tools/ab/base > $O/ab.json 2> $O/ab.err
echo "rc=$?" >> $O/done.txt
rm -f $O/c1.pcap
