#!/bin/bash
# tools/exp_sweep.sh <outdir> <name:VAR=val,VAR2=val>... -- one short bench per variant (GPU box).
# "name:" alone runs the default build; H264R_LIB=<path> selects a variant library.
# Every run has its own time limit; the sweep stops at the first failure.
set -e
OUT=$(realpath -m "$1"); shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
ARGS=${BENCH_ARGS:-"--steps 10 --warmup 2 --no-cpu --latency-pictures 0"}
mkdir -p "$OUT"
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  envargs=()
  IFS=',' read -ra kv <<< "$envs"
  for e in "${kv[@]}"; do [ -n "$e" ] && envargs+=("$e"); done
  echo "== $name ${envargs[*]}"
  env "${envargs[@]}" timeout -k 10 150 python3 "$ROOT/bench.py" $ARGS > "$OUT/$name.json" 2> "$OUT/$name.err"
  python3 - "$OUT/$name.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernel_ms"]
print(f"  {d['value']/1e6:8.1f} M MB/s  {d['ms_per_step']:.3f} ms/step  inter {k['inter']:.3f} intra {k['intra']:.3f} deblock {k['deblock']:.3f}  verified={d['verified_vs_oracle']}")
PY
done
