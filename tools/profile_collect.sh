#!/bin/bash
# Copy what tools/profile_round.sh left under gpurun_out/prof_<round>/ into profiles/<round>/.
set -eu
r=${1:-r01}
cd "$(dirname "$0")/.."
src=gpurun_out/prof_$r
dst=profiles/$r
mkdir -p "$dst"
cp "$src/bench.json" "$dst/bench.json"
cp "$(find "$src/trace" -name '*kernel_stats.csv' | head -1)" "$dst/kernel_stats.csv"
cp "$(find "$src/trace" -name '*domain_stats.csv' | head -1)" "$dst/domain_stats.csv"
cp "$src/pmc_hbm.csv" "$dst/pmc_hbm.csv"
[ -f "$src/pmc_mfma.csv" ] && cp "$src/pmc_mfma.csv" "$dst/pmc_mfma.csv"
[ -f "$src/stamps_gru.txt" ] && grep -v amdgpu.ids "$src/stamps_gru.txt" > "$dst/stamps_gru.txt"
[ -f "$src/stamps_dec.txt" ] && grep -v amdgpu.ids "$src/stamps_dec.txt" > "$dst/stamps_dec.txt"
grep -E "^(CPU\(s\)|Model name|Thread|Core|Socket)" "$src/host_cpu.txt" > "$dst/host_cpu.txt" || true
for f in "$src"/bench_*.json; do [ -f "$f" ] && cp "$f" "$dst/"; done
cat > "$dst/command.txt" <<TXT
# produced by tools/profile_round.sh $r on one MI355X (gpurun), collected by tools/profile_collect.sh
# bench line (driver command):             python bench.py
# kernel trace + stats (kernel_stats.csv):  rocprofv3 --kernel-trace --stats --output-format csv -d .../trace -o prof -- python bench.py --steps 10 --warmup 2 --no-cpu --no-pmc
# HBM traffic (pmc_hbm.csv), two passes:    rocprofv3 --pmc FETCH_SIZE --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu --no-kernel-timing --no-pmc --no-graph
#                                           rocprofv3 --pmc WRITE_SIZE --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu --no-kernel-timing --no-pmc --no-graph
# MFMA evidence (pmc_mfma.csv), one pass:   rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu --no-kernel-timing --no-pmc --no-graph
# per-phase stamps (stamps_*.txt):          python tools/gru_stamps.py; python tools/xdec_stamps.py
# secondary bench lines (bench_<config>.json): tools/bench_lines.sh (python bench.py --config <config>)
TXT
echo "collected $src -> $dst"
