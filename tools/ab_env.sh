#!/bin/bash
# tools/ab_env.sh <outdir> <config> <VAR=value>... -- bench.py A/B over environment settings
# of libh264r.so, one JSON line per setting ("-" = none), on one MI355X (GPU box); every run
# verifies its pictures against the oracle before timing (AB_ARGS adds bench arguments, e.g.
# --mode chain).
OUT=$1; CFG=$2; shift 2
mkdir -p "$OUT"
i=0
for E in "$@"; do
  if [ "$E" = "-" ]; then SET=(); else SET=("$E"); fi
  env "${SET[@]}" timeout -k 10 240 python bench.py --config $CFG --steps 10 --warmup 2 --no-cpu --latency-pictures 0 $AB_ARGS \
      > "$OUT/v$i.json" 2> "$OUT/v$i.err" || exit 1
  python -c "import json; d=json.loads(open('$OUT/v$i.json').read().strip().splitlines()[-1]); print('$E', 'config $CFG', 'Mmb/s %.1f' % (d['value']/1e6), 'ms %.2f' % d['ms_per_step'], 'kernels', d['kernel_ms'], 'verified', d['verified_vs_oracle'])"
  i=$((i+1))
done
