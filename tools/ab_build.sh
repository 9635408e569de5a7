#!/bin/bash
# Build the library of git revision REV (default HEAD) into seq2seq-attention-asr_amd/s2s_amd/ab/NAME.so
# from a clean worktree, for same-box A/B runs:  S2S_HIP_LIB=<that .so> python bench.py
set -eu
rev=${1:-HEAD}; name=${2:-base}
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" worktree add -q --detach "$tmp" "$rev"
make -C "$tmp/seq2seq-attention-asr_amd/csrc" -j8 >/dev/null
mkdir -p "$root/seq2seq-attention-asr_amd/s2s_amd/ab"
cp "$tmp/seq2seq-attention-asr_amd/s2s_amd/libs2s_hip.so" "$root/seq2seq-attention-asr_amd/s2s_amd/ab/$name.so"
git -C "$root" worktree remove --force "$tmp"
echo "built $rev -> seq2seq-attention-asr_amd/s2s_amd/ab/$name.so"
