#!/bin/bash
# tools/gpu_session_r3d.sh -- config 3 A/B: k_deblock3 (8 lanes per picture-row), the level
# kernel's grid (H264R_LVL_MARGIN 3 / 5 blocks per CU below the occupancy answer), k_inter4r at
# 5 waves/SIMD (varlib/iw5: 96 VGPRs + spills).
set -o pipefail
O=gpurun_out/r3d; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so
tools/ab_mix.sh $O/ab3 3 $L $L,H264R_DEBLOCK3=1 $L,H264R_LVL_MARGIN=3 $L,H264R_LVL_MARGIN=5 varlib/iw5/libh264r.so \
    $L $L,H264R_DEBLOCK3=1 $L,H264R_LVL_MARGIN=3 $L,H264R_LVL_MARGIN=5 varlib/iw5/libh264r.so > $O/ab3.txt 2>&1
echo "session rc=$?"
