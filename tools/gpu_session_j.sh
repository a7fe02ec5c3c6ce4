#!/bin/bash
# tools/gpu_session_j.sh -- k_deblock3 (8 lanes per picture-row): parity on the large-batch
# GPU tests, then a bench A/B against k_deblock2 (configs 3, 2, 4); W2 = k_deblock3 at 4 waves/SIMD (spills).
set -o pipefail
O=gpurun_out/r03_j; mkdir -p $O
M=arrow-h264_amd/lib/libh264r.so; W2=varlib/d3w4/libh264r.so
H264R_DEBLOCK3=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread -k "large_batch or pipelined or 1080p or picture_groups" > $O/gputest_d3.log 2>&1 &&
tools/ab_mix.sh $O/ab3 3 $M $M,H264R_DEBLOCK3=1 $W2,H264R_DEBLOCK3=1 $M > $O/ab3.txt 2>&1 &&
tools/ab_mix.sh $O/ab2 2 $M $M,H264R_DEBLOCK3=1 $W2,H264R_DEBLOCK3=1 > $O/ab2.txt 2>&1 &&
tools/ab_mix.sh $O/ab4 4 $M $M,H264R_DEBLOCK3=1 $W2,H264R_DEBLOCK3=1 > $O/ab4.txt 2>&1
