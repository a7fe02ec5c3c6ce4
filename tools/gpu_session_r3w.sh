#!/bin/bash
# tools/gpu_session_r3w.sh -- config 5 (64 pictures of 2160p) with k_deblock2 (H264R_DEBLOCK2_MIN=64)
# instead of k_deblock (the default below 192 pictures).
set -o pipefail
O=gpurun_out/r3w; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so
tools/ab_mix.sh $O/ab5 5 $L $L,H264R_DEBLOCK2_MIN=64 $L $L,H264R_DEBLOCK2_MIN=64 > $O/ab5.txt 2>&1
echo "session rc=$?"
