# round 6: the replay mempool's object stride (2,368 B, as a DPDK mempool object: this tree's default)
# against exactly the 2-KiB data room (--mbuf-stride 0), drop-in at 16 and 1 pipelines, 3 alternating rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_aa
mkdir -p $O
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pipeline.py > $O/tests.log 2>&1 &&
timeout -k 10 600 python3 tools/dropin_bench.py --ab-env "NB_EXTRA_ARGS=--mbuf-stride 0" > $O/ab.json 2> $O/ab.err
echo "rc=$?" >> $O/done.txt
