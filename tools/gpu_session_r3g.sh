#!/bin/bash
# tools/gpu_session_r3g.sh [outdir name] -- final measurement at HEAD: every GPU test, smoke(), the default
# bench line (config 3), rocprofv3 kernel stats, configs 2/4/5, PMC passes at batch 1024, a
# per-phase trace of k_deblock2 (trace build, arrow-h264_amd/lib_trace), the standalone decoder's
# wall time per frame on the 1080p CABAC stream with and without the overlapped picture end.
set -o pipefail
O=gpurun_out/${1:-r3g}; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err &&
tools/stats.sh $O/stats "--steps 5 --warmup 1 --no-cpu --no-verify --latency-pictures 0" &&
for c in 2 4 5; do
  timeout -k 10 300 python3 bench.py --config $c --cpu-seconds 4 > $O/bench_c$c.json 2> $O/bench_c$c.err || exit 1
done &&
tools/pmc.sh $O/pmc "--steps 2 --warmup 1 --no-cpu --no-verify --latency-pictures 0" > $O/pmc.txt 2>&1 &&
ST=tests/golden/streams/hp_1080p_cabac_ibbp_4slices.264 &&
timeout -k 10 120 arrow-h264_amd/lib/h264dec -i $ST -o $O/dec.yuv -r 10 > $O/h264dec_time.txt 2>&1 &&
H264P_SYNC=1 timeout -k 10 120 arrow-h264_amd/lib/h264dec -i $ST -o $O/dec.yuv -r 10 >> $O/h264dec_time.txt 2>&1 &&
rm -f $O/dec.yuv &&
H264R_LIB=arrow-h264_amd/lib_trace/libh264r.so timeout -k 10 180 python3 tools/trace_deblock.py 1024 8 > $O/trace_db2.txt 2>&1
echo "session rc=$?"
