"""Latency-chain probe (SURVEY 8(d) latency mode): the bench's dependent config-3 chain, one
picture per launch, run on its own so that `rocprofv3 --kernel-trace` sees only its kernels.

    python3 tools/latency_probe.py [pictures] [config]
    rocprofv3 --kernel-trace -d gpurun_out/lat -o lat -- python3 tools/latency_probe.py 64
    python3 tools/latency_probe.py --analyze gpurun_out/lat/.../lat_kernel_trace.csv

--analyze prints, per kernel, the mean duration per picture and the mean gap before it, and the
picture span (first kernel start to last kernel end), over the timed half of the chain."""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "arrow-h264_amd"))


def analyze(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    k = [(r["Kernel_Name"].split("(")[0], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    # pictures: a new picture starts at each k_inter4r
    pics, cur = [], []
    for e in k:
        if e[0].startswith("k_inter4r") and cur:
            pics.append(cur)
            cur = []
        cur.append(e)
    if cur:
        pics.append(cur)
    pics = pics[len(pics) // 2:]                  # the timed half
    from collections import defaultdict
    dur, gap = defaultdict(float), defaultdict(float)
    span = 0.0
    for p in pics:
        prev_end = None
        for name, s, e in p:
            dur[name] += (e - s) / 1e3
            if prev_end is not None:
                gap[name] += (s - prev_end) / 1e3
            prev_end = e
        span += (p[-1][2] - p[0][1]) / 1e3
    n = len(pics)
    print(f"{n} pictures; span per picture {span / n:.1f} us")
    for name in dur:
        print(f"  {name:24s} {dur[name] / n:8.1f} us   gap before {gap[name] / n:6.1f} us")
    starts = [p[0][1] for p in pics]
    if len(starts) > 1:
        print(f"picture period {(starts[-1] - starts[0]) / (len(starts) - 1) / 1e3:.1f} us")


def main():
    if sys.argv[1:2] == ["--analyze"]:
        return analyze(sys.argv[2])
    import torch
    import h264r
    from h264r import synth
    import bench
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    cfg_idx = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    L = h264r.lib()
    W, H = bench.CONFIG_SIZE[cfg_idx]
    cfg = synth.default_cfg(L, cfg_idx, W, H)
    refs = synth.refpics(L, cfg)
    dec = h264r.Decoder(0, W, H)
    cs = torch.cuda.Stream()
    with torch.cuda.stream(cs):
        ms, nl, ver = bench.latency_chain(dec, L, cfg, refs, cs.cuda_stream, n, 2)
    print(f"latency {ms:.3f} ms per picture over {nl} pictures, verified {ver}")


if __name__ == "__main__":
    main()
