#!/bin/bash
# tools/gpu_session_r3o.sh -- the walk (k_intra_pic) at 6 waves/SIMD (varlib/w6, -DH264R_WALK_WAVES=6:
# 79 VGPRs, 56 SGPRs spilled to VGPR lanes instead of 86 at 8 waves) against the library at
# 8, configs 2 and 3.
set -o pipefail
O=gpurun_out/r3o; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so; W=varlib/w6/libh264r.so
tools/ab_mix.sh $O/ab2 2 $L $W $L $W > $O/ab2.txt 2>&1 &&
tools/ab_mix.sh $O/ab3 3 $L $W > $O/ab3.txt 2>&1
echo "session rc=$?"
