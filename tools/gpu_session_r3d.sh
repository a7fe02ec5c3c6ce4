#!/bin/bash
# tools/gpu_session_r3d.sh -- every GPU test at the working tree (16-byte level-list entries
# with the record dwords, next entry prefetched), then config 3 A/B: HEAD (varlib/head) vs the
# working tree, k_deblock3 (8 lanes per picture-row), the level kernel's grid
# (H264R_LVL_MARGIN=3), k_inter4r at 5 waves/SIMD (varlib/iw5: 96 VGPRs + spills, HEAD tree).
set -o pipefail
O=gpurun_out/r3d; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so; H=varlib/head/libh264r.so
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 &&
tools/ab_mix.sh $O/ab3 3 $H $L $L,H264R_DEBLOCK3=1 $L,H264R_LVL_MARGIN=3 varlib/iw5/libh264r.so \
    $H $L $L,H264R_DEBLOCK3=1 $L,H264R_LVL_MARGIN=3 varlib/iw5/libh264r.so > $O/ab3.txt 2>&1 &&
tools/ab_mix.sh $O/ab4 4 $H $L $H $L > $O/ab4.txt 2>&1
echo "session rc=$?"
