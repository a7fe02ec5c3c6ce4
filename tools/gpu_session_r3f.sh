#!/bin/bash
# tools/gpu_session_r3f.sh -- every GPU test at the working tree (branch-free chroma MC with
# its six row loads in flight together; the workgroup LDS tables from loads issued
# together; the WP parameters of all planes in one batch), then A/B against HEAD
# (varlib/head) on configs 3, 4, 5.
set -o pipefail
O=gpurun_out/r3f; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so; H=varlib/head/libh264r.so
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 &&
tools/ab_mix.sh $O/ab3 3 $H $L $H $L > $O/ab3.txt 2>&1 &&
tools/ab_mix.sh $O/ab4 4 $H $L $H $L > $O/ab4.txt 2>&1 &&
tools/ab_mix.sh $O/ab5 5 $H $L > $O/ab5.txt 2>&1
echo "session rc=$?"
