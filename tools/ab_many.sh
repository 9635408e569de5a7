# Same-box A/B of several builds (ab/NAME.so for NAME in $AB_NAMES; env pairs NAME:VAR=VAL via AB_ENV_<NAME>),
# alternating, AB_ROUNDS rounds: gpurun_out/abm_NAME_ROUND.json
set -e
D=seq2seq-attention-asr_amd/s2s_amd/ab
for r in $(seq 1 ${AB_ROUNDS:-2}); do
  for v in $AB_NAMES; do
    lib=${v%%+*}
    envs=""
    [ "$v" != "$lib" ] && envs=${v#*+}
    env $envs S2S_HIP_LIB=$D/$lib.so timeout -k 10 200 python bench.py --no-cpu --no-pmc --no-kernel-timing --steps 40 > gpurun_out/abm_${v}_$r.json 2>/dev/null
  done
done
