#!/bin/bash
# tools/gpu_session_r3c.sh -- every GPU test at the working tree; A/B of the k_dbinfo single
# round-trip loads + slice headers in LDS + 8-wave walk (arrow-h264_amd/lib) against the
# previous commit (varlib/head) on configs 3, 2 and 4.
set -o pipefail
O=gpurun_out/r3c; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so; H=varlib/head/libh264r.so
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 &&
tools/ab_mix.sh $O/ab3 3 $H $L $H $L > $O/ab3.txt 2>&1 &&
tools/ab_mix.sh $O/ab2 2 $H $L $H $L > $O/ab2.txt 2>&1 &&
tools/ab_mix.sh $O/ab4 4 $H $L $H $L > $O/ab4.txt 2>&1
echo "session rc=$?"
