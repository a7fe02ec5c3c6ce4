#!/bin/bash
# tools/gpu_session_f.sh -- the deblocking records apart (H264R_DBINFO 1 / 2): GPU parity
# tests in both modes, then a bench A/B of 0 / 1 / 2 on configs 3, 4 and 2.
set -o pipefail
O=gpurun_out/r03_f; mkdir -p $O
H264R_DBINFO=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/gputest_db2.log 2>&1 &&
H264R_DBINFO=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread -k "1080p or batch" > $O/gputest_db1.log 2>&1 &&
tools/ab_env.sh $O/ab3 3 H264R_DBINFO=0 H264R_DBINFO=1 H264R_DBINFO=2 H264R_DBINFO=0 H264R_DBINFO=2 > $O/ab3.txt 2>&1 &&
tools/ab_env.sh $O/ab4 4 H264R_DBINFO=0 H264R_DBINFO=1 H264R_DBINFO=2 > $O/ab4.txt 2>&1 &&
tools/ab_env.sh $O/ab2 2 H264R_DBINFO=0 H264R_DBINFO=2 > $O/ab2.txt 2>&1
