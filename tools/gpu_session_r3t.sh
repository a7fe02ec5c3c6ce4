#!/bin/bash
# tools/gpu_session_r3t.sh -- every GPU test and smoke() with k_dbinfo at 8 groups per workgroup.
set -o pipefail
O=gpurun_out/${1:-r3t}; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
echo "session rc=$?"
