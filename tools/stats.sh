#!/bin/bash
# tools/stats.sh <outdir> [bench args] -- rocprofv3 kernel-trace stats of a short bench run (GPU box)
OUT=$(realpath -m "$1"); shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
ARGS=${*:-"--steps 3 --warmup 1 --no-cpu --no-verify --latency-pictures 0"}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# (k_intra_levels takes a plain launch by default: rocprofv3 7.2 crashes at exit after a cooperative one)
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/bench.log" 2>&1
