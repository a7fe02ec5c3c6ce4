#!/bin/bash
# tools/measure_r06.sh <outdir> -- PMC traffic of every config's launch sequence from this code
# (GPU box): config 3 at the headline batch (-> profiles/traffic.json), configs 2 / 4 / 5 with their
# N=1 lines and cpu_baseline (tools/measure_configs.sh), and config 5 in chain mode
# (-> profiles/traffic_c5_chain.json).
set -e
OUT=$(realpath -m "$1")
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
bash "$ROOT/tools/pmc.sh" "$OUT/pmc_c3" --steps 3 --warmup 1 --no-cpu --no-verify --latency-pictures 0
python3 "$ROOT/tools/pmc_summary.py" "$OUT/pmc_c3" --mbs $((1024 * 8160)) --config 3 --json "$OUT/traffic.json" > "$OUT/pmc_c3.txt"
echo "pmc c3 done"
bash "$ROOT/tools/pmc.sh" "$OUT/pmc_c5_chain" --mode chain --config 5 --steps 3 --warmup 1 --no-cpu --no-verify
python3 "$ROOT/tools/pmc_summary.py" "$OUT/pmc_c5_chain" --mbs $((32 * 32400)) --config 5 --json "$OUT/traffic_c5_chain.json" > "$OUT/pmc_c5_chain.txt"
echo "pmc c5 chain done"
bash "$ROOT/tools/measure_configs.sh" "$OUT" 2 4 5
