#!/bin/bash
# Build a libairice.so variant for tools/ab_table.py from a csrc directory:
#   tools/build_variant.sh <csrc_dir> <out.so> [extra hipcc flags...]
set -e
SRC=$1; OUT=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$SRC"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -mllvm -disable-machine-licm \
  -Wno-unused-result -I"$ROOT/include" -I. "$@" -shared -o "$OUT" \
  $(ls *.hip *.cpp | grep -v '^cli_')
