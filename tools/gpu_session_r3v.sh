#!/bin/bash
# tools/gpu_session_r3v.sh -- placement: config 3 with the batch and scratch shifted by pads of
# 0, 1, 3, 7, 64, 0 MB (H264R_BENCH_PAD_MB) on one box, against the box-to-box spread of k_deblock2.
set -o pipefail
O=gpurun_out/r3v; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so
tools/ab_mix.sh $O/pad 3 $L,H264R_BENCH_PAD_MB=0 $L,H264R_BENCH_PAD_MB=1 $L,H264R_BENCH_PAD_MB=3 $L,H264R_BENCH_PAD_MB=7 $L,H264R_BENCH_PAD_MB=64 $L,H264R_BENCH_PAD_MB=0 > $O/pad.txt 2>&1
echo "session rc=$?"
