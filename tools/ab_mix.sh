#!/bin/bash
# tools/ab_mix.sh <outdir> <config> <lib>[,VAR=value]... -- bench.py A/B over (library,
# environment) pairs on one MI355X (GPU box); every run verifies against the oracle.
OUT=$1; CFG=$2; shift 2
mkdir -p "$OUT"
i=0
for SPEC in "$@"; do
  LIB=${SPEC%%,*}; ENVS=(); [ "$SPEC" != "$LIB" ] && IFS=, read -ra ENVS <<< "${SPEC#*,}"
  env H264R_LIB=$LIB "${ENVS[@]}" timeout -k 10 240 python bench.py --config $CFG --steps 10 --warmup 2 --no-cpu \
      --latency-pictures 0 > "$OUT/v$i.json" 2> "$OUT/v$i.err" || exit 1
  python -c "import json; d=json.loads(open('$OUT/v$i.json').read().strip().splitlines()[-1]); print('$SPEC', 'config $CFG', 'Mmb/s %.1f' % (d['value']/1e6), 'ms %.2f' % d['ms_per_step'], 'kernels', d['kernel_ms'], 'verified', d['verified_vs_oracle'])"
  i=$((i+1))
done
