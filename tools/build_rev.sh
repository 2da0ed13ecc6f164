#!/bin/bash
# Build libdpt.so of a git revision's csrc (for A/Bs against HEAD without compile-time knobs):
#   bash tools/build_rev.sh <rev> <tag>  ->  dp-tokenization_amd/csrc/build/var_<tag>/libdpt.so
set -e
cd "$(dirname "$0")/.."
rev=$1; tag=$2
tmp=$(mktemp -d /tmp/dpt_rev_XXXX)
git archive "$rev" dp-tokenization_amd/csrc include | tar -x -C "$tmp"
out=$PWD/dp-tokenization_amd/csrc/build/var_$tag
mkdir -p "$out"
make -s -C "$tmp/dp-tokenization_amd/csrc" -j8 OUT="$out/libdpt.so" "$out/libdpt.so"
rm -rf "$tmp"
ls -la "$out/libdpt.so"
