set -o pipefail
mkdir -p gpurun_out
A=$PWD/seq2seq-attention-asr_amd/s2s_amd/ab
S2S_HIP_LIB=$A/base.so timeout -k 10 120 python tools/ab_bitwise.py save gpurun_out/ab_base.pt 2>&1 | grep -v amdgpu
S2S_HIP_LIB=$A/new.so timeout -k 10 120 python tools/ab_bitwise.py save gpurun_out/ab_new.pt 2>&1 | grep -v amdgpu
python tools/ab_bitwise.py cmp gpurun_out/ab_base.pt gpurun_out/ab_new.pt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_full.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gputest_full.log | grep -v "^    "; exit 1; }
tail -2 gpurun_out/gputest_full.log
timeout -k 10 300 python tools/ab_convlstm.py 2>&1 | grep -v amdgpu
