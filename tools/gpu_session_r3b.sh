#!/bin/bash
# tools/gpu_session_r3b.sh -- own-parser GPU tests; A/B of k_dbinfo packed strength stores
# (varlib/dbpack) and 8-waves/SIMD intra kernels (varlib/w8); PMC passes at batch 1024.
set -o pipefail
O=gpurun_out/r3b; mkdir -p $O
L=arrow-h264_amd/lib/libh264r.so
timeout -k 10 300 python -u -m pytest tests/test_parser.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest_parser.log 2>&1 &&
tools/ab_mix.sh $O/ab3 3 $L varlib/dbpack/libh264r.so varlib/w8/libh264r.so $L varlib/dbpack/libh264r.so varlib/w8/libh264r.so > $O/ab3.txt 2>&1 &&
tools/ab_mix.sh $O/ab2 2 $L varlib/w8/libh264r.so $L varlib/w8/libh264r.so > $O/ab2.txt 2>&1 &&
tools/pmc.sh $O/pmc "--steps 2 --warmup 1 --no-cpu --no-verify --latency-pictures 0" > $O/pmc.txt 2>&1
echo "session rc=$?"
