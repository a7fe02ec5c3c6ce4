#!/bin/bash
# tools/bench_configs.sh <outdir> -- N=1 bench lines + rocprofv3 kernel stats for SURVEY
# configs 2, 4 and 5 (config 3 is the default bench line).  GPU box.
set -e
OUT=$(realpath -m "$1")
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
for c in 2 4 5; do
  timeout -k 10 300 python3 "$ROOT/bench.py" --config $c --cpu-seconds 6 > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err"
  bash "$ROOT/tools/stats.sh" "$OUT/stats_c$c" --config $c --steps 3 --warmup 1 --no-cpu --no-verify --latency-pictures 0
done
echo configs done
