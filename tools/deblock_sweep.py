#!/usr/bin/env python3
"""GPU box: deblocking kernel time (h264r_last_timing phase 2) of the two schedules over batch
sizes, 1080p config 3 pictures -- the data behind H264R_DEBLOCK2_MIN's default."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "arrow-h264_amd"))
import torch  # noqa: E402,F401
import h264r  # noqa: E402
from h264r import _abi as A, batch as B, synth  # noqa: E402

L = h264r.lib()
W, H = 120, 68
cfg = synth.default_cfg(L, 3, W, H)
base = [synth.picture(L, cfg, i) for i in range(8)]
refs = synth.refpics(L, cfg)
sizes = [int(a) for a in sys.argv[1:]] or [1, 8, 32, 64, 128, 256, 512, 1024]
with h264r.Decoder(0, W, H) as dec:
    for s, (y, u, v) in enumerate(refs):
        dec.set_ref(s, y, u, v)
    dec.set_timing(True)
    for n in sizes:
        host = B.pack([base[i % 8] for i in range(n)], h264r.quant_flat())
        db = B.to_device(host, n, None)
        row = []
        for flag in (A.DBG_DEBLOCK_MB, A.DBG_DEBLOCK_ROWS):
            dec.set_debug(flag)
            best = 1e9
            for _ in range(3):
                dec.decode_batch(db.batch)
                dec.check()
                best = min(best, dec.last_timing()[2])
            row.append(best)
        dec.set_debug(0)
        print(f"{n:5d} pictures: k_deblock {row[0]:8.3f} ms  k_deblock2 {row[1]:8.3f} ms  ratio {row[0] / row[1]:5.2f}", flush=True)
