#!/bin/bash
# tools/gpu_session_r3j.sh -- the walk's band height: k_intra_pic with 8 (HEAD), 4 and 2 MB rows
# per band (varlib/r4, varlib/r2: -DH264R_WALK_ROWS; a band's rows start 2 MBs apart and the
# workgroup holds its slot until its last row ends, so a band of R rows idles 2(R-1) of
# 120 + 2(R-1) steps), configs 2 and 3; then k_deblock2's per-ticket trace (lib_trace).
set -o pipefail
O=gpurun_out/r3j; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so; A=varlib/r4/libh264r.so; B=varlib/r2/libh264r.so
tools/ab_mix.sh $O/ab2 2 $L $A $B $L $A $B > $O/ab2.txt 2>&1 &&
tools/ab_mix.sh $O/ab3 3 $L $A $B > $O/ab3.txt 2>&1 &&
H264R_LIB=arrow-h264_amd/lib_trace/libh264r.so timeout -k 10 180 python3 tools/trace_deblock.py 1024 8 > $O/trace_db2.txt 2>&1
echo "session rc=$?"
