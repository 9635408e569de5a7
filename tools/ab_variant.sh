#!/bin/bash
# Build the working tree's library with extra compiler flags into seq2seq-attention-asr_amd/s2s_amd/ab/NAME.so
# (same-box A/B of compile-time variants):  tools/ab_variant.sh NAME "-DFOO -DBAR"
set -eu
name=$1; extra=${2:-}
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
mkdir -p "$tmp/a" && cp -r "$root/seq2seq-attention-asr_amd/csrc" "$tmp/a/csrc"
rm -rf "$tmp/a/csrc/build"
mkdir -p "$tmp/include" "$root/seq2seq-attention-asr_amd/s2s_amd/ab"
cp "$root/include/s2s_hip.h" "$tmp/include/"
make -C "$tmp/a/csrc" -j8 EXTRA="$extra" OUT="$root/seq2seq-attention-asr_amd/s2s_amd/ab/$name.so" >/dev/null
rm -rf "$tmp"
echo "built $name ($extra)"
