#!/bin/bash
# tools/gpu_session_r3h.sh -- every GPU test at the working tree, then A/B on configs 3, 2, 4:
#   head   = varlib/head (k_dbinfo round-trip commit 9a50834)
#   noskip = + branch-free chroma MC (six row loads in flight together), the LDS tables from
#            loads issued together, the WP parameters of all planes in one batch
#   lib    = + k_inter4r leaving all-intra groups before its LDS fill (H264R_INTER_SKIP)
set -o pipefail
O=gpurun_out/r3h; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so; N=varlib/noskip/libh264r.so; H=varlib/head/libh264r.so
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 &&
tools/ab_mix.sh $O/ab3 3 $H $N $L $H $N $L > $O/ab3.txt 2>&1 &&
tools/ab_mix.sh $O/ab2 2 $H $N $L $H $N $L > $O/ab2.txt 2>&1 &&
tools/ab_mix.sh $O/ab4 4 $H $N $L $H $N $L > $O/ab4.txt 2>&1
echo "session rc=$?"
