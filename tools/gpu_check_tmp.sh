set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_full.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gputest_full.log | grep -v "^    "; exit 1; }
tail -2 gpurun_out/gputest_full.log
timeout -k 10 300 python tools/ab_convlstm.py 2>&1 | grep -v amdgpu
