#!/bin/bash
# tools/measure_configs.sh <outdir> [configs...] -- the off-headline measurement set (GPU box):
# for each SURVEY config an N=1 bench line with cpu_baseline, then tools/pmc.sh over the same
# workload (kernel stats + PMC passes) summarised to <outdir>/traffic_c<N>.json; and the
# config-3 line at SURVEY 8(d)'s default batch of 64 pictures beside the 1024-picture headline.
set -e
OUT=$(realpath -m "$1"); shift
CFGS=${*:-"2 4 5"}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
declare -A MBS=([2]=$((1024 * 8160)) [3]=$((1024 * 8160)) [4]=$((256 * 8160)) [5]=$((64 * 32400)))
timeout -k 10 300 python3 "$ROOT/bench.py" --config 3 --batch 64 --cpu-seconds 6 > "$OUT/bench_c3_b64.json" 2> "$OUT/bench_c3_b64.err"
echo "c3 b64 done"
for c in $CFGS; do
  timeout -k 10 300 python3 "$ROOT/bench.py" --config $c --cpu-seconds 6 > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err"
  echo "bench c$c done"
  bash "$ROOT/tools/pmc.sh" "$OUT/pmc_c$c" --config $c --steps 3 --warmup 1 --no-cpu --no-verify --latency-pictures 0
  python3 "$ROOT/tools/pmc_summary.py" "$OUT/pmc_c$c" --mbs ${MBS[$c]} --config $c --json "$OUT/traffic_c$c.json" > "$OUT/pmc_c$c.txt"
  echo "pmc c$c done"
done
echo "measure done"
