#!/bin/bash
# tools/gpu_check.sh <tag> [what...] -- one GPU-box session (run through gpurun): the GPU tests,
# smoke, the default bench, the chain-mode lines of configs 5 and 4 at one GPU, the throughput
# lines of configs 2, 4 and 5, and a rocprofv3
# kernel-stats run of the default bench.  Every GPU step has its own time limit and the steps are
# chained with &&: the session stops at the first failure.  Outputs under gpurun_out/<tag>/.
set -o pipefail
T=${1:?tag}; shift
WHAT=${*:-"tests smoke bench chain5 chain4 c2 c4 c5 prof"}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
run() { echo "== $1 $(date +%T)"; }
has() { [[ " $WHAT " == *" $1 "* ]]; }
set -e
if has tests; then run tests
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > $O/gputest.log 2>&1
  tail -3 $O/gputest.log; fi
if has smoke; then run smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; tail -1 $O/smoke.log; fi
if has bench; then run bench
  timeout -k 10 400 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err; tail -c 400 $O/bench_c3.json; echo; fi
if has chain5; then run chain5
  timeout -k 10 400 python bench.py --mode chain --config 5 --steps 10 > $O/chain_c5.json 2> $O/chain_c5.err; tail -c 300 $O/chain_c5.json; echo; fi
if has chain4; then run chain4
  timeout -k 10 400 python bench.py --mode chain --config 4 --steps 10 > $O/chain_c4.json 2> $O/chain_c4.err; tail -c 300 $O/chain_c4.json; echo; fi
for c in 2 4 5; do if has c$c; then run c$c
  timeout -k 10 400 python bench.py --config $c --no-cpu --latency-pictures 0 > $O/bench_c$c.json 2> $O/bench_c$c.err; tail -c 300 $O/bench_c$c.json; echo; fi; done
if has prof; then run prof
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu --latency-pictures 0 > $GRAFT_REPO_ROOT/$O/prof_bench.json 2> $GRAFT_REPO_ROOT/$O/prof.err
  cd $GRAFT_REPO_ROOT; find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \; ; head -12 $O/kernel_stats.csv | cut -c1-120; fi
echo "== done $(date +%T)"
