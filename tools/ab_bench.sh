#!/bin/bash
# Same-box A/B: alternate bench.py runs over the libraries named on the command line
# (seq2seq-attention-asr_amd/s2s_amd/ab/<name>.so), ROUNDS times each; one summary line per run.
set -eu
cd "$(dirname "$0")/.."
rounds=${ROUNDS:-3}
for r in $(seq "$rounds"); do
  for name in "$@"; do
    out=$(S2S_HIP_LIB="$PWD/seq2seq-attention-asr_amd/s2s_amd/ab/$name.so" timeout -k 10 200 python bench.py --no-cpu --steps ${STEPS:-20} ${BENCH_ARGS:-} 2>/dev/null | tail -1)
    python -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1], d['ms_per_step'], {k: round(v['us_per_step']) for k, v in d['kernels'].items()})" "$name" "$out"
  done
done
