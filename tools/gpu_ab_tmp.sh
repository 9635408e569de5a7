set -o pipefail
A=$PWD/seq2seq-attention-asr_amd/s2s_amd/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_full.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gputest_full.log | grep -v "^    "; exit 1; }
tail -1 gpurun_out/gputest_full.log
for r in 1 2; do for v in base new; do
  echo -n "$v: "; S2S_HIP_LIB=$A/$v.so AB_ONLY=graph timeout -k 10 120 python tools/ab_convlstm.py 2>&1 | grep -v amdgpu || exit 1
done; done
