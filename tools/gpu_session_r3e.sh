#!/bin/bash
# tools/gpu_session_r3e.sh -- config 3 batch-size sweep (k_deblock2 rounds: 1024 pictures =
# 544 (group, row) waves per XCD over 256 slots = 2.125 rounds; 960 = 510 = 1.99)
set -o pipefail
O=gpurun_out/r3e; mkdir -p $O
tools/ab_batch.sh $O/b3 3 1024 960 896 1088 1024 960 896 1088 > $O/batch3.txt 2>&1
echo "session rc=$?"
