#!/bin/bash
# tools/gpu_session_i.sh -- the new defaults (k_dbinfo + k_inter4r at 4 waves/SIMD, residual
# loads after the MC, all-intra pictures to the walk): every GPU test, the default bench,
# rocprof kernel stats, a k_deblock2 trace and the PMC passes of config 3.
set -o pipefail
O=gpurun_out/r03_i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
tools/stats.sh $O/stats --steps 5 --warmup 1 --no-cpu --no-verify --latency-pictures 0 &&
H264R_LIB=varlib/trace/libh264r.so timeout -k 10 200 python tools/trace_deblock.py 1024 8 > $O/trace_db2_1024.txt 2>&1 &&
tools/pmc.sh $O/pmc3 --config 3 --batch 256 --steps 3 --warmup 1 --no-cpu --no-verify --latency-pictures 0 &&
H264R_LIB=varlib/trace_intra/libh264r.so timeout -k 10 200 python tools/trace_intra.py 120 2 > $O/trace_intra_c2.txt 2>&1
