set -o pipefail
ROUNDS=3 STEPS=20 bash tools/ab_bench.sh base new 2>&1 | cut -c1-120
