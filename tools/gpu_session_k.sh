#!/bin/bash
# tools/gpu_session_k.sh -- config 5 (2160p, 64 pictures: below the row walk's threshold):
# k_deblock vs the row walks at a lower threshold; then the diagnostics of session j.
set -o pipefail
O=gpurun_out/r03_k; mkdir -p $O
M=arrow-h264_amd/lib/libh264r.so
tools/ab_mix.sh $O/ab5 5 $M $M,H264R_DEBLOCK2_MIN=32 $M,H264R_DEBLOCK2_MIN=32,H264R_DEBLOCK3=1 > $O/ab5.txt 2>&1
