#!/bin/bash
# tools/gpu_session_r3s.sh -- groups per workgroup: k_inter4r with 2 consecutive 16-MB groups
# (varlib/g2, -DH264R_INTER_GROUPS=2: 6 VGPRs spilled, the LDS tables filled once per two
# groups), k_dbinfo with 2 or 8 instead of 4 (varlib/d2, varlib/d8): config 3 (and 4 for g2).
set -o pipefail
O=gpurun_out/r3s; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so
tools/ab_mix.sh $O/ab3 3 $L varlib/g2/libh264r.so varlib/d2/libh264r.so varlib/d8/libh264r.so $L varlib/g2/libh264r.so varlib/d2/libh264r.so varlib/d8/libh264r.so > $O/ab3.txt 2>&1 &&
tools/ab_mix.sh $O/ab4 4 $L varlib/g2/libh264r.so $L varlib/g2/libh264r.so > $O/ab4.txt 2>&1
echo "session rc=$?"
