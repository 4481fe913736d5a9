#!/bin/bash
# Round 3: where the ring's per-batch time settles: 4,096-batch runs (slope per eighth), in place and
# read only, C++ producer.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for v in ip ro; do timeout -k 10 200 tools/ring_bench $v 4096 || exit 1; done
