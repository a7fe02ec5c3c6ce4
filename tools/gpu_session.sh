#!/bin/bash
# tools/gpu_session.sh <tag> -- one GPU-box session (each step time-limited, chained with &&):
#   1. the GPU tests touched by recent changes;  2. bench A/B over the batch pipeline depth
#   (configs 3 and 4);  3. rocprofv3 kernel stats of the default bench.
set -o pipefail
T=$1; O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 180 --timeout-method thread \
    -k "pipelined or large_batch or 1080p or expired or lossless or b_explicit or sp" > $O/gputest.log 2>&1 &&
tools/ab_pipes.sh $O/pipes3 3 > $O/pipes3.txt 2>&1 &&
tools/ab_pipes.sh $O/pipes4 4 > $O/pipes4.txt 2>&1 &&
tools/stats.sh $O/stats "--steps 5 --warmup 1 --no-cpu --no-verify --latency-pictures 0"
