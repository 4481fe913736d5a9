# host-path tests (direct path completion word, stalled enqueue), drop-in sweep, kernel traces of nb_maglev --loop
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_d
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pipeline.py tests/test_gpu_zerocopy.py tests/test_gpu_parity.py > $O/tests.log 2>&1 &&
timeout -k 10 300 python3 tools/dropin_bench.py --extra > $O/dropin.json 2> $O/dropin.err &&
python3 tools/dropin_bench.py --write-pcap /tmp/c1.pcap &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt1 -o run -- netbricks_amd/host/nb_maglev --rx /tmp/c1.pcap --backends 65 --loop 2000000 --pipelines 1 > $O/kt1.json 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt16 -o run -- netbricks_amd/host/nb_maglev --rx /tmp/c1.pcap --backends 65 --loop 500000 --pipelines 16 > $O/kt16.json 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt16z -o run -- netbricks_amd/host/nb_maglev --rx /tmp/c1.pcap --backends 65 --loop 300000 --pipelines 16 --zero-copy 1 > $O/kt16z.json 2>&1
echo "rc=$?" >> $O/done.txt
