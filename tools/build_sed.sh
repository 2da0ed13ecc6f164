#!/bin/bash
# Build libdpt.so of the working tree's csrc with one sed expression applied to dpt_kernels.hip (A/Bs of
# a constant without a compile-time knob in the source):
#   bash tools/build_sed.sh <tag> '<sed expression>'  ->  dp-tokenization_amd/csrc/build/var_<tag>/libdpt.so
set -e
cd "$(dirname "$0")/.."
tag=$1; expr=$2
tmp=$(mktemp -d /tmp/dpt_sed_XXXX)
mkdir -p "$tmp/dp-tokenization_amd" && cp -r dp-tokenization_amd/csrc "$tmp/dp-tokenization_amd/" && cp -r include "$tmp/"
rm -rf "$tmp/dp-tokenization_amd/csrc/build"
sed -i -e "$expr" "$tmp/dp-tokenization_amd/csrc/dpt_kernels.hip"
diff -q dp-tokenization_amd/csrc/dpt_kernels.hip "$tmp/dp-tokenization_amd/csrc/dpt_kernels.hip" > /dev/null && { echo "sed changed nothing"; exit 1; }
out=$PWD/dp-tokenization_amd/csrc/build/var_$tag
mkdir -p "$out"
make -s -C "$tmp/dp-tokenization_amd/csrc" -j8 OUT="$out/libdpt.so" "$out/libdpt.so"
rm -rf "$tmp"
ls -la "$out/libdpt.so"
