#!/bin/bash
# tools/gpu_session_r3x.sh -- rocprofv3 kernel stats of configs 2, 4, 5 at the end-of-round HEAD.
set -o pipefail
O=gpurun_out/r3x; mkdir -p $O
for c in 2 4 5; do
  tools/stats.sh $O/c$c "--config $c --steps 5 --warmup 1 --no-cpu --no-verify --latency-pictures 0" || exit 1
done
echo "session rc=$?"
