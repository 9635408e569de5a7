set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_graph.py tests/test_gpu_ragged.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gputest.log | grep -v "^    "; exit 1; }
tail -2 gpurun_out/gputest.log
ROUNDS=3 STEPS=20 bash tools/ab_bench.sh base new 2>&1 | cut -c1-200
timeout -k 10 120 python tools/xdec_stamps.py > gpurun_out/xdec_new.txt 2>&1; grep -v amdgpu gpurun_out/xdec_new.txt
for n in base new; do S2S_HIP_LIB=$PWD/seq2seq-attention-asr_amd/s2s_amd/ab/$n.so timeout -k 10 200 python bench.py --config librispeech_vgg_b16 --no-cpu --no-pmc --no-kernel-timing --steps 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('vgg $n', d['ms_per_step'])"; done
