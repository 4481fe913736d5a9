# round 6: 24-B header windows (this tree) against 32-B windows (commit c49d932's library, built by
# tools/build_ab.sh into tools/ab/w32), drop-in at 16 and 1 pipelines, 3 alternating rounds on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_v
mkdir -p $O
timeout -k 10 600 python3 tools/dropin_bench.py --ab-lib tools/ab/w32 > $O/ab.json 2> $O/ab.err
echo "rc=$?" >> $O/done.txt
