#!/bin/bash
# tools/gpu_ab.sh <tag> <configs> <lib|->... -- A/B of variant libraries (H264R_LIB; "-" = the
# default lib/) on one GPU box: one short bench per (config, library), each verified against
# the oracle before timing.  Outputs under gpurun_out/<tag>/.
set -o pipefail
T=${1:?tag}; CFGS=${2:?configs}; shift 2
O=gpurun_out/$T
mkdir -p $O
for c in $CFGS; do
  i=0
  for L in "$@"; do
    if [ "$L" = "-" ]; then LIB=arrow-h264_amd/lib/libh264r.so; else LIB=$L; fi
    H264R_LIB=$LIB timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu --latency-pictures 0 \
        > $O/c${c}_v$i.json 2> $O/c${c}_v$i.err || { echo "FAIL $L config $c"; tail -5 $O/c${c}_v$i.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/c${c}_v$i.json').read().strip().splitlines()[-1]); k=d['kernel_ms']; print('%-40s c%d %7.1f Mmb/s  %6.2f ms  inter %.2f intra %.2f deblock %.2f  verified %s' % ('$L', $c, d['value']/1e6, d['ms_per_step'], k['inter'], k['intra'], k['deblock'], d['verified_vs_oracle']))" | tee -a $O/summary.txt
    i=$((i+1))
  done
done
