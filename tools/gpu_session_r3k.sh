#!/bin/bash
# tools/gpu_session_r3k.sh -- intra prediction loops unrolled and branch-free (I_4x4 steps with
# per-slot wave-uniform block parameters, I_8x8 reference filter as one (A + 2B + C + 2) >> 2
# form with taps from an e[]-ordered copy, chroma DC by selects): every GPU test, then A/B
# against HEAD (varlib/head) on configs 2, 3, 4, with the walk's band height as a second
# factor (varlib/r4, varlib/r2: -DH264R_WALK_ROWS=4 / 2 on the new code; a band's rows start
# 2 MBs apart and the workgroup holds its slot until its last row ends); then k_deblock2's
# per-ticket trace (lib_trace).
set -o pipefail
O=gpurun_out/r3k; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so; H=varlib/head/libh264r.so; A=varlib/r4/libh264r.so; B=varlib/r2/libh264r.so
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 &&
tools/ab_mix.sh $O/ab2 2 $H $L $A $B $H $L $A $B > $O/ab2.txt 2>&1 &&
tools/ab_mix.sh $O/ab3 3 $H $L $A $H $L $A > $O/ab3.txt 2>&1 &&
tools/ab_mix.sh $O/ab4 4 $H $L > $O/ab4.txt 2>&1 &&
H264R_LIB=arrow-h264_amd/lib_trace/libh264r.so timeout -k 10 180 python3 tools/trace_deblock.py 1024 8 > $O/trace_db2.txt 2>&1
echo "session rc=$?"
