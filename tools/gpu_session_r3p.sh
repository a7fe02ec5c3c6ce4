#!/bin/bash
# tools/gpu_session_r3p.sh -- k_inter4r's chroma MC with both planes' rows loaded before either is
# used (one global round trip instead of two): every GPU test, then A/B against HEAD
# (varlib/head) on configs 3 and 4.
set -o pipefail
O=gpurun_out/r3p; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so; H=varlib/head/libh264r.so
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 &&
tools/ab_mix.sh $O/ab3 3 $H $L $H $L > $O/ab3.txt 2>&1 &&
tools/ab_mix.sh $O/ab4 4 $H $L $H $L > $O/ab4.txt 2>&1
echo "session rc=$?"
