# round 4, last check of the in-tree library the driver will load: every GPU test and smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_last
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "rc=$?" >> $O/done.txt
