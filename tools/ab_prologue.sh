# A/B of the decoder-fold placement (S2S_PROLOGUE, capi.cpp model_step_impl) on one GPU
set -e
for m in 0 1 2; do
  S2S_PROLOGUE=$m timeout -k 10 200 python bench.py --no-cpu --no-pmc --steps 40 > gpurun_out/ab_$m.json 2>/dev/null
done
