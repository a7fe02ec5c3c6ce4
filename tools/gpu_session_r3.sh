#!/bin/bash
# tools/gpu_session_r3.sh <tag> -- HEAD check on one GPU box (each step time-limited, chained
# with &&): every GPU test, smoke(), the default bench line, configs 2/4/5, rocprofv3 stats.
set -o pipefail
T=$1; O=gpurun_out/$T
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err &&
tools/stats.sh $O/stats "--steps 5 --warmup 1 --no-cpu --no-verify --latency-pictures 0" &&
for c in 2 4 5; do
  timeout -k 10 300 python3 bench.py --config $c --cpu-seconds 4 > $O/bench_c$c.json 2> $O/bench_c$c.err || exit 1
done
echo session done
