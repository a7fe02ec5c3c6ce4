#!/bin/bash
# tools/gpu_session_r3r.sh -- k_intra_levels at 7 waves/SIMD (varlib/l7, -DH264R_LVL_WAVES=7: 72
# VGPRs, none spilled; 6 waves at 77 VGPRs in the library): configs 3 and 4.
set -o pipefail
O=gpurun_out/r3r; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so; V=varlib/l7/libh264r.so
tools/ab_mix.sh $O/ab3 3 $L $V $L $V > $O/ab3.txt 2>&1 &&
tools/ab_mix.sh $O/ab4 4 $L $V $L $V > $O/ab4.txt 2>&1
echo "session rc=$?"
