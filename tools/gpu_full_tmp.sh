set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_full.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gputest_full.log | grep -v "^    "; exit 1; }
tail -2 gpurun_out/gputest_full.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_default.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_default.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
