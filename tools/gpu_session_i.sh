#!/bin/bash
# tools/gpu_session_i.sh -- every GPU test at the new defaults, the default bench, rocprof
# kernel stats, then k_deblock3 (H264R_DEBLOCK3=1) parity on the large-batch tests and a
# bench A/B against k_deblock2 (configs 3, 2, 4).
set -o pipefail
O=gpurun_out/r03_i; mkdir -p $O
M=arrow-h264_amd/lib/libh264r.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
tools/stats.sh $O/stats --steps 5 --warmup 1 --no-cpu --no-verify --latency-pictures 0 &&
H264R_DEBLOCK3=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread -k "large_batch or pipelined or 1080p or picture_groups" > $O/gputest_d3.log 2>&1 &&
tools/ab_mix.sh $O/ab3 3 $M $M,H264R_DEBLOCK3=1 $M > $O/ab3.txt 2>&1 &&
tools/ab_mix.sh $O/ab2 2 $M $M,H264R_DEBLOCK3=1 > $O/ab2.txt 2>&1 &&
tools/ab_mix.sh $O/ab4 4 $M $M,H264R_DEBLOCK3=1 > $O/ab4.txt 2>&1
