set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 200 python tools/ab_graph_knob.py s2s_debug_gru_ring 1 0 7 > gpurun_out/ab_ring.txt 2>&1 && cat gpurun_out/ab_ring.txt
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ringpmc/pmc_$c -o pmc -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu --no-kernel-timing --no-pmc --no-graph > /dev/null 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT && python tools/pmc_table.py gpurun_out/ringpmc > gpurun_out/ringpmc/pmc_hbm.csv && head -5 gpurun_out/ringpmc/pmc_hbm.csv
timeout -k 10 120 python tools/gru_stamps.py > gpurun_out/ring_stamps.txt 2>&1 && cat gpurun_out/ring_stamps.txt
