#!/bin/bash
# tools/pmc.sh -- rocprofv3 kernel stats + PMC passes over a short bench run (GPU box).
# One counter group per rocprofv3 run (gfx950 slot limits, MI355X_MICROARCH.md).
# usage: tools/pmc.sh <outdir> [bench args...]
set -e
OUT=$(realpath -m "$1"); shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
ARGS=${*:-"--batch 64 --steps 3 --warmup 1 --no-cpu --no-verify --latency-pictures 0"}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# (k_intra_levels takes a plain launch by default: rocprofv3 7.2 crashes at exit after a cooperative one)
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/stats.log" 2>&1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/pmc$i.log" 2>&1
done
echo "pmc done"
