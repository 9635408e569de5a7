#!/bin/bash
# Round profile artifacts, run on a GPU box:  tools/profile_round.sh r01  ->  gpurun_out/prof_r01/
#   bench.json        the default bench line (driver command: python bench.py)
#   trace/            rocprofv3 --kernel-trace --stats of a 10-step bench run (kernel_stats, domain_stats)
#   pmc_hbm.csv       HBM bytes per dispatch from two --pmc passes (FETCH_SIZE, WRITE_SIZE) of an eager run
# then copy the summaries into profiles/<round>/ (tools/profile_collect.sh).
set -eu
r=${1:-r01}
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/gpurun_out/prof_$r
rm -rf "$out"
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 python "$root/bench.py" > "$out/bench.json"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o prof -- \
  python "$root/bench.py" --steps 10 --warmup 2 --no-cpu --no-pmc > "$out/trace_bench.json"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$out/pmc_$c" -o pmc -- \
    python "$root/bench.py" --steps 2 --warmup 1 --no-cpu --no-kernel-timing --no-pmc --no-graph > /dev/null
done
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d "$out/pmc_MFMA" -o pmc -- \
  python "$root/bench.py" --steps 2 --warmup 1 --no-cpu --no-kernel-timing --no-pmc --no-graph > /dev/null
python "$root/tools/pmc_table.py" "$out" > "$out/pmc_hbm.csv"
python "$root/tools/pmc_table.py" --mfma "$out" > "$out/pmc_mfma.csv"
# per-phase latency breakdown of the persistent recurrences (in-kernel s_memrealtime stamps)
timeout -k 10 120 python "$root/tools/gru_stamps.py" > "$out/stamps_gru.txt" 2>&1
timeout -k 10 120 python "$root/tools/xdec_stamps.py" > "$out/stamps_dec.txt" 2>&1
lscpu > "$out/host_cpu.txt"
