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
grep -E "^(CPU\(s\)|Model name|Thread|Core|Socket)" "$src/host_cpu.txt" > "$dst/host_cpu.txt" || true
cat > "$dst/command.txt" <<TXT
# produced by tools/profile_round.sh $r on one MI355X (gpurun), collected by tools/profile_collect.sh
# bench line (driver command):             python bench.py
# kernel trace + stats (kernel_stats.csv):  rocprofv3 --kernel-trace --stats --output-format csv -d .../trace -o prof -- python bench.py --steps 10 --warmup 2 --no-cpu --no-pmc
# HBM traffic (pmc_hbm.csv), two passes:    rocprofv3 --pmc FETCH_SIZE --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu --no-kernel-timing --no-pmc --no-graph
#                                           rocprofv3 --pmc WRITE_SIZE --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu --no-kernel-timing --no-pmc --no-graph
TXT
echo "collected $src -> $dst"
