set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gputest.log | grep -v "^    "; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 300 python tools/ab_vgg.py s2s_debug_gemm_lt 1 0 3 > gpurun_out/ab_vgg_lt.txt 2>&1; cat gpurun_out/ab_vgg_lt.txt
