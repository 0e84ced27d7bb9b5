#!/bin/bash
# Build a variant of libnexg.so with extra compiler defines, for in-process
# A/B runs (tools/bench_malformed.py --libs, tools/bench_ser_ab.py):
#   bash tools/build_variant.sh abtmp/libnexg_tpw4.so -DNEXG_PING_TPW=4
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
out=$(realpath -m "$1"); shift
mkdir -p "$(dirname "$out")"
tmp=$(mktemp -d)
mkdir -p "$tmp/a/b" && cp -r "$ROOT/nex_amd/csrc" "$tmp/a/b/csrc" && cp -r "$ROOT/include" "$tmp/a/include"
rm -rf "$tmp/a/b/csrc/build"
make -s -C "$tmp/a/b/csrc" -j8 LIB="$out" HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $*"
rm -rf "$tmp"
echo "built $out"
