#!/bin/bash
# tools/gpu_session_g.sh -- PMC passes (tools/pmc.sh) of config 3 and config 2 at batch 256
set -o pipefail
O=gpurun_out/r03_g; mkdir -p $O
tools/pmc.sh $O/c3 --config 3 --batch 256 --steps 3 --warmup 1 --no-cpu --no-verify --latency-pictures 0 &&
tools/pmc.sh $O/c2 --config 2 --batch 256 --steps 3 --warmup 1 --no-cpu --no-verify --latency-pictures 0
