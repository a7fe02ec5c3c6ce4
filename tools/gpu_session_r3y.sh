#!/bin/bash
# tools/gpu_session_r3y.sh -- k_inter4r skips the pictures k_dbinfo found no inter or I_PCM MB in
# (per-picture counts in the launch's sync words): every GPU test, then A/B against HEAD
# (varlib/head) on configs 2 and 3.
set -o pipefail
O=gpurun_out/r3y; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so; H=varlib/head/libh264r.so
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 &&
tools/ab_mix.sh $O/ab2 2 $H $L $H $L > $O/ab2.txt 2>&1 &&
tools/ab_mix.sh $O/ab3 3 $H $L $H $L > $O/ab3.txt 2>&1
echo "session rc=$?"
