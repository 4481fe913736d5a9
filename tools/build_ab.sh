#!/bin/bash
# Build libnbgpu.so of a git revision into tools/ab/lib_<name>.so (A/B timing in one GPU call).
# usage: [EXTRA=-DFLAG] tools/build_ab.sh <name> [<rev>]   (no rev: the working tree)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REV=$2
OUT=$ROOT/tools/ab/lib_$NAME.so
mkdir -p "$ROOT/tools/ab"
T=$(mktemp -d)
if [ -z "$REV" ]; then
  tar -C "$ROOT" -cf - netbricks_amd/csrc include | tar -x -C "$T"
else
  git -C "$ROOT" archive "$REV" netbricks_amd/csrc include | tar -x -C "$T"
fi
rm -f "$T"/netbricks_amd/csrc/*.o
make -C "$T/netbricks_amd/csrc" -s OUT="$OUT" EXTRA="$EXTRA"
rm -rf "$T"
echo "built $OUT"
