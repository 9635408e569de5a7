# Same-box A/B of two builds of libs2s_hip.so (S2S_HIP_LIB): ab/old.so vs ab/new.so, alternating
set -e
D=seq2seq-attention-asr_amd/s2s_amd/ab
R=${AB_ROUNDS:-2}
for r in $(seq 1 $R); do
  for v in old new; do
    S2S_HIP_LIB=$D/$v.so timeout -k 10 200 python bench.py --no-cpu --no-pmc --no-kernel-timing --steps 40 > gpurun_out/ab_${v}_$r.json 2>/dev/null
  done
done
