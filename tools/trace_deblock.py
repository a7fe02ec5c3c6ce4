#!/usr/bin/env python3
"""Diagnostic (GPU box): per-wave timing of the deblocking walk from a trace build,
    make -C arrow-h264_amd OBJ=build_trace LIBDIR=lib_trace EXTRA=-DH264R_TRACE
    H264R_LIB=arrow-h264_amd/lib_trace/libh264r.so python tools/trace_deblock.py [pictures] [flag] [band] [lpu]
(flag 8 = k_deblock2, 4 = k_deblock, 128 = the split walk's luma and chroma kernels) [band = the build's H264R_DB2_BAND, lpu = its H264R_DB2_LPU].  k_deblock2 records
per ticket (a band of MB rows of a picture group) {start, end} in 100 MHz ticks and the core
cycles of its four phases summed over the walk."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "arrow-h264_amd"))
import torch  # noqa: E402,F401
import h264r  # noqa: E402
from h264r import batch as B, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
flag = int(sys.argv[2]) if len(sys.argv) > 2 else 8
band = int(sys.argv[3]) if len(sys.argv) > 3 else 4
lpu = int(sys.argv[4]) if len(sys.argv) > 4 else 8      # the build's H264R_DB2_LPU (lanes per unit)
L = h264r.lib()
W, H = 120, 68
cfg = synth.default_cfg(L, 3, W, H)
pics = [synth.picture(L, cfg, i % 8) for i in range(n)]
refs = synth.refpics(L, cfg)
out = os.path.join(tempfile.mkdtemp(), "tr.bin")
with h264r.Decoder(0, W, H) as dec:
    for s, (y, u, v) in enumerate(refs):
        dec.set_ref(s, y, u, v)
    host = B.pack(pics, h264r.quant_flat())
    dec.set_debug(flag)
    for it in range(3):                       # the last launch is the one traced
        db = B.to_device(host, n, None)
        if it == 2:
            os.environ["H264R_TRACE_OUT"] = out
        dec.decode_batch(db.batch)
        dec.check()
if flag == 4:
    # k_deblock: per ticket (pair-major: ticket = pair * n + pic) {start, first step, end,
    # polling ticks} in 100 MHz ticks, then core cycles of: tile assembly, vertical pass,
    # horizontal pass (with the rows above), write-back + ring + carry -- summed over the
    # walk's W + 1 steps
    t = np.fromfile(out, np.uint64).reshape(-1, 8).astype(np.int64)
    k = n * ((H + 1) // 2)
    t = t[:k]
    t0 = t[:, 0].min()
    start, end = (t[:, 0] - t0) / 100.0, (t[:, 2] - t0) / 100.0
    print(f"{n} pictures, {k} waves: kernel span {end.max():.0f} us; wave duration mean {np.mean(end - start):.0f} us")
    steps = W + 1
    print(f"polling share {np.mean(t[:, 3] / np.maximum(t[:, 2] - t[:, 0], 1)):.3f}; "
          f"us per step {np.mean((t[:, 2] - t[:, 1]) / 100.0 / steps):.2f}")
    print("cycles per step (assemble, V pass, H pass, write-back):", np.round(t[:, 4:8].mean(0) / steps, 0))
    for p in (0, 1, k // n // 2, k // n - 1):
        sel = np.arange(k) // n == p
        print(f"pair {p:3d}: start {start[sel].mean():8.1f} us end {end[sel].mean():8.1f} us, poll "
              f"{t[sel, 3].mean() / 100.0:8.1f} us, cycles/step {np.round(t[sel, 4:8].mean(0) / steps, 0)}")
    sys.exit(0)
suffixes = [".2y", ".2c"] if flag == 128 else [".2"]   # the split walk's luma / chroma kernels
def report(t):

    units = 64 // lpu
    ng = (n + units // band - 1) // (units // band)
    nb = (H + band - 1) // band
    k = ng * nb
    steps = W + band + 2
    t = t[:k]
    t0 = t[:, 0].min()
    start, end = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0       # microseconds
    print(f"{n} pictures, {k} waves ({nb} bands of {band} rows x {ng} groups): kernel span {end.max():.0f} us; "
          f"wave duration mean {np.mean(end - start):.0f} us ({np.mean(end - start) / steps:.2f} us/step), "
          f"start spread {start.min():.0f}..{start.max():.0f} us")
    ph = t[:, 2:6].astype(np.float64)
    tot = ph.sum(1, keepdims=True)
    print("phase share (V, record wait, stores + staging + fill, H + publish + fetch):", np.round((ph / tot).mean(0), 3))
    print("cycles per step by phase:", np.round(ph.mean(0) / steps, 0))
    bands = np.arange(k) // ng
    for r in sorted(set((0, 1, 2, nb // 2, nb - 1))):
        sel = bands == r
        print(f"band {r:3d}: start {start[sel].mean():8.1f} us end {end[sel].mean():8.1f} us, wait share "
              f"{(ph[sel, 1] / tot[sel, 0]).mean():.3f}, cycles/step by phase {np.round(ph[sel].mean(0) / steps, 0)}")
    hist = np.histogram(start, bins=10)
    print("wave starts (us) histogram:", hist[0].tolist(), np.round(hist[1], 0).tolist())


for sfx in suffixes:
    print(f"== {sfx}")
    report(np.fromfile(out + sfx, np.uint64).reshape(-1, 8).astype(np.int64))
