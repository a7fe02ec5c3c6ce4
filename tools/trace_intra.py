#!/usr/bin/env python3
"""Diagnostic: per-MB latency trace of k_intra_levels and the walk k_intra_pic (lib built
with -DH264R_TRACE_INTRA):
    H264R_LIB=<trace lib> python tools/trace_intra.py [pictures] [config]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "arrow-h264_amd"))
import torch  # noqa: E402,F401
import h264r  # noqa: E402
from h264r import batch as B, synth  # noqa: E402

L = h264r.lib()
W, H, n = 120, 68, int(sys.argv[1]) if len(sys.argv) > 1 else 256
config = int(sys.argv[2]) if len(sys.argv) > 2 else 3
cfg = synth.default_cfg(L, config, W, H)
pics = [synth.picture(L, cfg, i) for i in range(n)]
refs = synth.refpics(L, cfg)
dec = h264r.Decoder(0, W, H)
for s, (y, u, v) in enumerate(refs):
    dec.set_ref(s, y, u, v)
db = B.to_device(B.pack(pics, h264r.quant_flat()), n, None)
dec.decode_batch(db.batch)
dec.check()
out = np.zeros((1 << 20, 4), np.uint64)
cnt = C.c_uint(0)
L.h264r_trace_intra_dump(out.ctypes.data_as(C.c_void_p), C.byref(cnt))
t = out[: cnt.value]
t0 = t[:, 0].astype(np.int64)
dur = (t[:, 1].astype(np.int64) - t0) / 100.0     # us (100 MHz)
walk = ((t[:, 2] >> 31) & 1).astype(bool) & ((t[:, 2] >> 32) == 0)
lvl = np.where(walk, -1, (t[:, 2] >> 32).astype(np.int64))
typ = np.where(walk, (t[:, 2] & 0xFF).astype(np.int64), (t[:, 2] & 0xFFFFFFFF).astype(np.int64))
wait = np.where(walk, ((t[:, 2] >> 8) & 0xFFFFF).astype(np.int64) / 100.0, 0.0)
start = (t0 - t0.min()) / 100.0
print("MBs", cnt.value, "walk MBs", int(walk.sum()))
if walk.any():
    print(f"walk: span {(start[walk] + dur[walk]).max():.1f} us, per MB {dur[walk].mean():.2f} us of which waiting for "
          f"the row above {wait[walk].mean():.2f} us")
for Lv in np.unique(lvl):
    m = lvl == Lv
    print(f"level {Lv}: n={m.sum()} start {start[m].min():.1f}..{start[m].max():.1f} us  end {(start[m] + dur[m]).max():.1f}  dur mean {dur[m].mean():.2f} p50 {np.median(dur[m]):.2f} max {dur[m].max():.2f}")
ph = np.stack([((t[:, 3] >> (16 * k)) & 0xFFFF).astype(np.int64) * 16 for k in range(4)], 1)   # core cycles
for ty in np.unique(typ):
    m = typ == ty
    print(f"type {ty}: n={m.sum()} dur mean {dur[m].mean():.2f} p50 {np.median(dur[m]):.2f}  "
          f"cycles to record / residual / tiles / prediction: {np.round(ph[m].mean(0), 0)}")
