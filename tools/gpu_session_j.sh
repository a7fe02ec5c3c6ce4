#!/bin/bash
# tools/gpu_session_j.sh -- diagnostics: k_deblock2 trace at 1024 pictures, PMC passes of
# config 3 (batch 256), the intra walk's per-MB trace on config 2.
set -o pipefail
O=gpurun_out/r03_j; mkdir -p $O
H264R_LIB=varlib/trace/libh264r.so timeout -k 10 200 python tools/trace_deblock.py 1024 8 > $O/trace_db2_1024.txt 2>&1 &&
tools/pmc.sh $O/pmc3 --config 3 --batch 256 --steps 3 --warmup 1 --no-cpu --no-verify --latency-pictures 0 &&
H264R_LIB=varlib/trace_intra/libh264r.so timeout -k 10 200 python tools/trace_intra.py 120 2 > $O/trace_intra_c2.txt 2>&1
