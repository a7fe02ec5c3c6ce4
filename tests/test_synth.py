"""Workload generator: deterministic, identical through both libraries, and the
SURVEY 8(d) distributions / byte accounting hold."""
import numpy as np
import pytest

import _oracle as O
import h264r
from h264r import _abi as A
from h264r import synth


def test_deterministic_and_same_in_product_and_oracle_lib():
    h264r.build()
    Lp, Lo = h264r.lib(), O.lib()
    for cidx in (2, 3, 4):
        cp = synth.default_cfg(Lp, cidx, 20, 12)
        co = synth.default_cfg(Lo, cidx, 20, 12)
        a, b = synth.picture(Lp, cp, 3), synth.picture(Lo, co, 3)
        assert synth.input_digest(a) == synth.input_digest(b)
        assert synth.input_digest(a) == synth.input_digest(synth.picture(Lp, cp, 3))
        assert synth.input_digest(a) != synth.input_digest(synth.picture(Lp, cp, 4))


@pytest.mark.parametrize("cidx", [2, 3, 4, 5])
def test_distributions(cidx):
    L = O.lib()
    cfg = synth.default_cfg(L, cidx, 120, 68)
    p = synth.picture(L, cfg, 0)
    t = p.mbs["mb_type"]
    intra = (p.mbs["flags"] & A.MBF_INTRA) != 0
    if cidx == 2:
        assert intra.all()
        for ty, lo, hi in ((A.I_4x4, .35, .45), (A.I_8x8, .35, .45), (A.I_16x16, .15, .25)):
            assert lo < np.mean(t == ty) < hi
    else:
        assert .07 < intra.mean() < .13
    assert ((p.mbs["qp_y"] >= 20) & (p.mbs["qp_y"] <= 40)).all()
    assert len(p.slices) == {2: 1, 3: 1, 4: 4, 5: 8}[cidx]
    if cidx >= 4:
        assert (p.slices["deblock_idc"] == 2).all() and (p.slices["wp_mode"] == 2).all()
    # unused lists carry ref -1 and a zero MV
    assert (p.mv[p.ref_idx < 0] == 0).all()
    # all 16 quarter-pel phases occur in inter pictures
    if cidx != 2:
        used = p.ref_idx[0] >= 0
        mx = (p.mv[0][used] & 0xFFFF).astype(np.int16) & 3
        my = (p.mv[0][used] >> 16).astype(np.int16) & 3
        assert len(set(zip(mx.tolist(), my.tolist()))) == 16


def test_algo_bytes_formula():
    L = O.lib()
    cfg = synth.default_cfg(L, 3, 16, 8)
    p = synth.picture(L, cfg, 0)
    r, w = synth.algo_bytes(L, p)
    assert w == 384 * 16 * 8
    # a fully coded P MB costs R = 32 + 4*128 + 16 + 256 + 80 + 384 = 1280 (SURVEY 8(d) + chroma DC)
    assert 32 * 128 < r < 1400 * 128


def test_level_block_sizes_match_offsets():
    from h264r.mbview import level_count
    L = O.lib()
    cfg = synth.default_cfg(L, 4, 22, 18, pcm_permille=30)
    p = synth.picture(L, cfg, 1)
    offs = p.mbs["coef_off"].astype(np.int64)
    sizes = np.array([level_count(m) for m in p.mbs])
    assert (offs[1:] == offs[:-1] + sizes[:-1]).all()
