#!/bin/bash
# Build libnbgpu.so of a git revision into tools/ab/lib_<name>.so (A/B timing in one GPU call).
# usage: tools/build_ab.sh <name> [<rev>]   (no rev: the working tree)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REV=$2
OUT=$ROOT/tools/ab/lib_$NAME.so
if [ -z "$REV" ]; then
  make -C "$ROOT/netbricks_amd/csrc" -s && cp "$ROOT/netbricks_amd/libnbgpu.so" "$OUT"
else
  T=$(mktemp -d); git -C "$ROOT" archive "$REV" netbricks_amd/csrc include | tar -x -C "$T"
  make -C "$T/netbricks_amd/csrc" -s OUT="$OUT"; rm -rf "$T"
fi
echo "built $OUT"
