set -o pipefail
A=$PWD/seq2seq-attention-asr_amd/s2s_amd/ab
for r in 1 2; do for v in base new; do
  echo -n "$v: "; S2S_HIP_LIB=$A/$v.so AB_ONLY=graph timeout -k 10 120 python tools/ab_convlstm.py 2>&1 | grep -v amdgpu || exit 1
done; done
