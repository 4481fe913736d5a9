# round 6: the producer's admission check kept until its next enqueue (this tree's nb_maglev) against
# checking all 65 queues every scheduler round (HEAD's nb_maglev in tools/ab/hostbase), drop-in at 16 and
# 1 pipelines, 3 alternating rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_z
mkdir -p $O
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pipeline.py > $O/tests.log 2>&1 &&
timeout -k 10 600 python3 tools/dropin_bench.py --ab-bin tools/ab/hostbase/nb_maglev > $O/ab.json 2> $O/ab.err
echo "rc=$?" >> $O/done.txt
