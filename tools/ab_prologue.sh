set -e
for m in 0 1 2; do
  S2S_PROLOGUE=$m timeout -k 10 200 python bench.py --no-cpu --no-pmc --steps 40 > gpurun_out/ab_$m.json 2>/dev/null
done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
