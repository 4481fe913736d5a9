# round 5, last check of the committed tree (with the compact kernel's XCD order): GPU suite and smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_x2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "rc=$?" >> $O/done.txt
