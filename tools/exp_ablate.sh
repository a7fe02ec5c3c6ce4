#!/bin/bash
# tools/exp_ablate.sh <outdir> -- k_inter4 ablation timings (GPU box): each explib/<variant>/libh264r.so
# (built with -DH264R_EXP_NO_LUMA / _NO_CHROMA / _NO_RES / _NO_DBINFO: measurement-only, wrong output)
# is swapped in and the config-3 bench is run (unverified unless VERIFY=' '); the per-kernel HIP-event
# times are kept.  VARIANTS lists the explib/ builds to run, in order (A/B pairs alternate).
set -e
OUT=$(realpath -m "$1"); mkdir -p "$OUT"
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cp "$ROOT/arrow-h264_amd/lib/libh264r.so" "$OUT/libh264r.so.keep"
i=0
for v in ${VARIANTS:-BASE NO_LUMA NO_CHROMA NO_RES NO_DBINFO}; do
  i=$((i+1))
  cp "$ROOT/explib/$v/libh264r.so" "$ROOT/arrow-h264_amd/lib/libh264r.so"
  timeout -k 10 200 python3 "$ROOT/bench.py" --no-cpu ${VERIFY:---no-verify} --steps ${STEPS:-5} --latency-pictures 0 > "$OUT/$i.$v.json" 2> "$OUT/$i.$v.err" || true
done
cp "$OUT/libh264r.so.keep" "$ROOT/arrow-h264_amd/lib/libh264r.so"
echo ablations done
