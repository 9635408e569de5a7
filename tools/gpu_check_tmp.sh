set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_frontend.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 300 python tools/ab_vgg.py s2s_debug_sconv_wgrad_implicit 1 0 3 > gpurun_out/ab_vgg.txt 2>&1; cat gpurun_out/ab_vgg.txt
