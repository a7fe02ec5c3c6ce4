#!/usr/bin/env python3
"""Debug helper (GPU box): where the GPU's SP reconstruction differs from the oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "arrow-h264_amd"))
import numpy as np
import _oracle as O
import h264r
from h264r import synth
L = h264r.lib()
dec = h264r.Decoder(0, 32, 32)
for sw in (0, 1):
    for qs in (0, 3, 5):
        cfg = synth.default_cfg(L, 3, 11, 9, sp_slices=1, intra_permille=0)
        p = synth.picture(L, cfg, 0)
        p.slices["sp_switch"][:] = sw; p.slices["qs_y"][:] = qs; p.slices["qs_c"][:] = qs
        refs = synth.refpics(L, cfg)
        got = dec.decode_picture(p, refs, no_deblock=True)
        want = O.decode(p, refs, stage="recon")
        d = got[0].astype(int) - want[0].astype(int)
        bad = np.argwhere(d != 0)
        print(f"sw={sw} qs={qs}: Y {len(bad)} differ; U {int((got[1]!=want[1]).sum())} V {int((got[2]!=want[2]).sum())}")
        if len(bad):
            y, x = bad[0]
            mb = (y // 16) * 11 + x // 16
            m = p.mbs[mb]
            print("  first", (x, y), "MB", mb, "type", m["mb_type"], "cbp", m["cbp"], "qp", m["qp_y"], "gpu", got[0][y, x], "want", want[0][y, x])
            blk = np.zeros((4, 4), int)
            for yy, xx in bad:
                if (yy // 16) * 11 + xx // 16 == mb:
                    blk[(yy % 16) // 4, (xx % 16) // 4] += 1
            print("  per 4x4 block of that MB:\n", blk)
            print("  gpu rows:\n", got[0][y - y % 16:y - y % 16 + 4, x - x % 16:x - x % 16 + 8])
            print("  want rows:\n", want[0][y - y % 16:y - y % 16 + 4, x - x % 16:x - x % 16 + 8])
