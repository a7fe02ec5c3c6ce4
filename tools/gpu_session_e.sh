#!/bin/bash
# tools/gpu_session_e.sh -- GPU tests of the current library, then a bench A/B of
# compile-time variants (tools/ab_lib.sh) on configs 3, 4 and 2.
set -o pipefail
O=gpurun_out/r03_e; mkdir -p $O
LIBS="arrow-h264_amd/lib/libh264r.so varlib/notile/libh264r.so varlib/head/libh264r.so"
timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py tests/test_stream_parity.py -m gpu -x -v --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 &&
tools/ab_lib.sh $O/ab3 3 $LIBS > $O/ab3.txt 2>&1 &&
tools/ab_lib.sh $O/ab4 4 $LIBS > $O/ab4.txt 2>&1 &&
tools/ab_lib.sh $O/ab2 2 $LIBS > $O/ab2.txt 2>&1
