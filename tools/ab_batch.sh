#!/bin/bash
# tools/ab_batch.sh <outdir> <config> <batch>... -- bench.py over batch sizes (pictures per
# step) on one MI355X, one line per run, every run verified against the oracle (GPU box).
OUT=$1; CFG=$2; shift 2
mkdir -p "$OUT"
i=0
for B in "$@"; do
  timeout -k 10 240 python bench.py --config $CFG --batch $B --steps 10 --warmup 2 --no-cpu --latency-pictures 0 \
      > "$OUT/v$i.json" 2> "$OUT/v$i.err" || exit 1
  python -c "import json; d=json.loads(open('$OUT/v$i.json').read().strip().splitlines()[-1]); print('batch $B', 'config $CFG', 'Mmb/s %.1f' % (d['value']/1e6), 'ms %.2f' % d['ms_per_step'], 'kernels', d['kernel_ms'], 'verified', d['verified_vs_oracle'])"
  i=$((i+1))
done
