#!/bin/bash
# tools/gpu_session_r3l.sh -- k_inter4r without its lane-divergent branch trees (the quarter-
# phase output pick by a 64-bit table and masks, dequant as one 4x4 / 8x8 form, plain / bi
# combine and WP parameters by selects, chroma DC arithmetic) and the intra taps / I_4x4 DC by
# masks: every GPU test, then A/B against HEAD (varlib/head) on configs 3, 2, 4, 5.
set -o pipefail
O=gpurun_out/r3l; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so; H=varlib/head/libh264r.so
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 &&
tools/ab_mix.sh $O/ab3 3 $H $L $H $L > $O/ab3.txt 2>&1 &&
tools/ab_mix.sh $O/ab2 2 $H $L > $O/ab2.txt 2>&1 &&
tools/ab_mix.sh $O/ab4 4 $H $L $H $L > $O/ab4.txt 2>&1 &&
tools/ab_mix.sh $O/ab5 5 $H $L > $O/ab5.txt 2>&1
echo "session rc=$?"
