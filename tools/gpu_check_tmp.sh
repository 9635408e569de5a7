set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_frontend.py -m gpu -x -q --timeout 200 --timeout-method thread -k "graph_step" > gpurun_out/gputest.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gputest.log | grep -v "^    "; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 120 python tools/diag_graph_tmp.py interleave 2>&1 | grep -v amdgpu
timeout -k 10 300 python tools/ab_convlstm.py 2>&1 | grep -v amdgpu
