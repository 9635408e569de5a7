#!/bin/bash
# Secondary bench lines of a round, run on a GPU box:  tools/bench_lines.sh r02  ->  gpurun_out/prof_r02/bench_*.json
# (config 2 is the default line of tools/profile_round.sh); tools/profile_collect.sh copies them to profiles/<round>/.
set -eu
r=${1:-r01}
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/gpurun_out/prof_$r
mkdir -p "$out"
cd /tmp
for c in timit_chorowski_dropout_b64 librispeech_chorowski_b32 librispeech_vgg_b16 timit_ragged_b32; do
  timeout -k 10 400 python "$root/bench.py" --config $c > "$out/bench_$c.json"
done
