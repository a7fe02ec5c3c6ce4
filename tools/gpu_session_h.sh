#!/bin/bash
# tools/gpu_session_h.sh -- k_inter4 occupancy A/B (residual loads after the motion
# compensation, 4 waves/SIMD for k_inter4r) and a k_deblock2 trace at 1024 pictures.
set -o pipefail
O=gpurun_out/r03_h; mkdir -p $O
M=arrow-h264_amd/lib/libh264r.so
V=(varlib/reslate3/libh264r.so varlib/reslate4/libh264r.so)
tools/ab_mix.sh $O/ab3 3 $M ${V[0]} ${V[1]},H264R_DBINFO=1 ${V[1]},H264R_DBINFO=2 $M,H264R_DBINFO=1 $M > $O/ab3.txt 2>&1 &&
tools/ab_mix.sh $O/ab4 4 $M ${V[0]} ${V[1]},H264R_DBINFO=1 ${V[1]},H264R_DBINFO=2 > $O/ab4.txt 2>&1 &&
H264R_LIB=varlib/trace/libh264r.so timeout -k 10 200 python tools/trace_deblock.py 1024 8 > $O/trace_db2_1024.txt 2>&1
