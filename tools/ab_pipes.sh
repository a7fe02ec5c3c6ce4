#!/bin/bash
# tools/ab_pipes.sh <outdir> [config] -- bench.py A/B over the batch pipeline depth (H264R_PIPES,
# h264r_host.hip run_batch) on one MI355X; one JSON line per setting (GPU box)
OUT=$1; CFG=${2:-3}
mkdir -p "$OUT"
for p in 1 2 3 4; do
  H264R_PIPES=$p timeout -k 10 240 python bench.py --config $CFG --steps 10 --warmup 2 --no-cpu --latency-pictures 0 \
      > "$OUT/pipes$p.json" 2> "$OUT/pipes$p.err" || exit 1
  python -c "import json,sys; d=json.loads(open('$OUT/pipes$p.json').read().strip().splitlines()[-1]); print('pipes', $p, 'Mmb/s %.1f' % (d['value']/1e6), 'ms %.2f' % d['ms_per_step'], 'kernels', d['kernel_ms'], 'verified', d['verified_vs_oracle'])"
done
