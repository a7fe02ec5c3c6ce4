#!/bin/bash
# tools/gpu_session_r3i.sh -- where config 2's walk (k_intra_pic) spends its time: PMC passes
# at batch 256 (VALU / wait / LDS per wave) and the per-MB trace of the walk (trace build
# varlib/tintra, -DH264R_TRACE_INTRA, 32 pictures: phase cycles and the wait for the row above).
set -o pipefail
O=gpurun_out/r3i; mkdir -p $O
tools/pmc.sh $O/pmc2 "--config 2 --batch 256 --steps 2 --warmup 1 --no-cpu --no-verify --latency-pictures 0" > $O/pmc2.txt 2>&1 &&
H264R_LIB=varlib/tintra/libh264r.so timeout -k 10 180 python3 tools/trace_intra.py 32 2 > $O/trace_c2.txt 2>&1
echo "session rc=$?"
