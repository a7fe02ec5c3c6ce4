"""Per-macroblock views of a canonical picture (the unit Decoder.decode takes)."""
from __future__ import annotations

import numpy as np

from . import _abi as A


def level_count(rec, chroma_format: int = 1) -> int:
    """int16 entries of one MB's compacted level block (include/h264r.h; 4:2:2: 8 chroma blocks
    and 8 DC levels per plane, a PCM MB 512 samples; 4:4:4: three luma-like blocks, a PCM MB
    3 x 256 samples)."""
    if int(rec["mb_type"]) == A.I_PCM:
        return {0: 128, 2: 256, 3: 384}.get(chroma_format, 192)
    cbpl, cbpc = int(rec["cbp"]) & 15, int(rec["cbp"]) >> 4
    if chroma_format in (0, 3):                       # 4:0:0: the luma block alone
        return (3 if chroma_format == 3 else 1) * (64 * bin(cbpl).count("1") + (16 if int(rec["mb_type"]) == A.I_16x16 else 0))
    nb = 8 if chroma_format == 2 else 4                 # chroma 4x4 blocks per plane
    n = 64 * bin(cbpl).count("1")
    n += 32 * nb if cbpc == 2 else 0
    n += 16 if int(rec["mb_type"]) == A.I_16x16 else 0
    n += 2 * nb if cbpc else 0
    return n


def iter_mbs(p):
    """Yield (addr, record[1], levels, mv[2,16], ref_idx[2,16]) in raster order."""
    W, H = p.cfg.width_mbs, p.cfg.height_mbs
    mv = p.mv.reshape(2, H, 4, W, 4).transpose(1, 3, 0, 2, 4).reshape(H, W, 2, 16)
    rr = p.ref_idx.reshape(2, H, 4, W, 4).transpose(1, 3, 0, 2, 4).reshape(H, W, 2, 16)
    for a in range(W * H):
        rec = p.mbs[a:a + 1].copy()
        off = int(rec["coef_off"][0])
        lv = p.levels[off:off + level_count(rec[0], A.idc_of(p.cfg.chroma_format))]
        yield a, rec, lv, np.ascontiguousarray(mv[a // W, a % W]), np.ascontiguousarray(rr[a // W, a % W])
