#!/bin/bash
# tools/gpu_session_r3u.sh -- k_dbinfo at 16 groups per workgroup (varlib/d16) against 8 (lib): configs 3 and 4.
set -o pipefail
O=gpurun_out/r3u; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so; V=varlib/d16/libh264r.so
tools/ab_mix.sh $O/ab3 3 $L $V $L $V > $O/ab3.txt 2>&1 &&
tools/ab_mix.sh $O/ab4 4 $L $V > $O/ab4.txt 2>&1
echo "session rc=$?"
