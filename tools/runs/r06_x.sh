# round 6: the host-batch server's per-batch timeline (tools/runs/mk_hrprobe.sh's measurement build via
# LD_LIBRARY_PATH): nb_maglev --loop at 1, 4 and 16 pipelines, 64 blocks, then the stamps' summary
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_x
mkdir -p $O
python3 tools/dropin_bench.py --write-pcap $O/c1.pcap &&
for p in 1 4 16; do
  LD_LIBRARY_PATH=$PWD/tools/ab/hrprobe NBG_PROBE_OUT=$O/p$p.bin timeout -k 10 120 netbricks_amd/host/nb_maglev --rx $O/c1.pcap --backends 65 --batch 992 --loop 3000000 --pipelines $p --host-ring 64 > $O/p$p.json 2> $O/p$p.err || break
  python3 tools/hrprobe_stats.py $O/p$p.bin > $O/p$p.stats || break
done
echo "rc=$?" >> $O/done.txt
rm -f $O/c1.pcap
