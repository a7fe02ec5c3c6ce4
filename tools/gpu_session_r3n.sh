#!/bin/bash
# tools/gpu_session_r3n.sh -- deblocking without lane-divergent branch trees: k_deblock2's hand-off
# pair offsets from a 64-bit table, k_deblock's line filter with every candidate computed and
# selected and its decisions as bitwise ANDs.  Every GPU test, then A/B against HEAD
# (varlib/head): config 3 (k_deblock2), config 5 (k_deblock), and the latency chain (k_deblock).
set -o pipefail
O=gpurun_out/r3n; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so; H=varlib/head/libh264r.so
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 &&
tools/ab_mix.sh $O/ab3 3 $H $L $H $L > $O/ab3.txt 2>&1 &&
tools/ab_mix.sh $O/ab5 5 $H $L $H $L > $O/ab5.txt 2>&1 &&
for v in $H $L $H $L; do
  H264R_LIB=$v timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-verify >> $O/latency.jsonl 2>> $O/latency.err || exit 1
  echo "$v $(tail -1 $O/latency.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["latency"])')" >> $O/latency.txt
done
echo "session rc=$?"
