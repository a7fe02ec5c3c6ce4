"""4:4:4 pictures (chroma_format_idc 3) on the GPU path against the oracle.

A 4:4:4 picture codes every colour plane like luma (decode_one_component for PLANE_Y / U / V,
decoder.cc:65-79; luma-style deblocking of Cb and Cr, deblock.cc:422).  The library decodes it as
three 4:2:0-shaped launch sequences of the same kernels, plane pl in the luma slots
(h264r_host.hip run_444, k_derive444).  The oracle is pinned to the compiled reference on 4:4:4
pictures by the golden fixtures (tests/golden/golden.json, the *444* cases, also run by
test_gpu_parity.py); these tests add batches under every deblocking schedule, per-picture DPB
tables, a slice band, the streaming API keeping a picture as a reference, and the refusals.
Bit-exact on every sample.
"""
import numpy as np
import pytest

import _oracle as O
import h264r
from h264r import _abi as A
from h264r import batch as B
from h264r import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    h264r.build()
    return h264r.lib()


@pytest.fixture(scope="module")
def dec(L):
    d = h264r.Decoder(0, 240, 135, chroma_format=3)
    yield d
    d.close()


DEBLOCKS = (A.DBG_DEBLOCK_MB, A.DBG_DEBLOCK_ROWS, A.DBG_DEBLOCK_SPLIT)


def _diff(a, b):
    bad = np.argwhere(a != b)
    return None if not len(bad) else f"{len(bad)} samples differ, first at (y, x) = {tuple(bad[0])}"


def _batch(dec, pics, refs, deblocks=DEBLOCKS, rows=None):
    for s, (y, u, v) in enumerate(refs):
        dec.set_ref(s, y, u, v)
    want = [O.decode(p, refs) for p in pics]
    host = B.pack(pics, h264r.quant_flat())
    H = pics[0].cfg.height_mbs
    r0, r1 = rows if rows else (0, H)
    for db_flag in deblocks:
        db = B.to_device(host, len(pics), None)
        dec.set_debug(db_flag)
        try:
            dec.decode_batch(db.batch, rows=rows)
            dec.check()
        finally:
            dec.set_debug(0)
        for i in range(len(pics)):
            got = db.planes(i)
            for k in range(3):
                d = _diff(got[k][r0 * 16:r1 * 16], want[i][k][r0 * 16:r1 * 16])
                assert d is None, f"deblock flag {db_flag} picture {i} plane {k}: {d}"


@pytest.mark.parametrize("cidx,W,H,n,over", [
    (2, 22, 9, 3, dict(pcm_permille=30)),
    (3, 22, 9, 4, dict(num_refs=2)),
    (3, 22, 9, 3, dict(wp_mode=1, num_refs=3, intra_permille=250, pcm_permille=20)),
    (4, 22, 9, 4, dict(num_refs=4)),
    (4, 22, 9, 3, dict(wp_mode=1, num_refs=4, num_slices=3, deblock_idc=2)),
    (3, 11, 9, 3, dict(qp_min=0, qp_max=20, lossless_permille=500)),
    (4, 120, 17, 2, dict()),                                     # 1080p-wide
])
def test_gpu_444_batches(L, dec, cidx, W, H, n, over):
    cfg = synth.default_cfg(L, cidx, W, H, chroma_format=3, **over)
    _batch(dec, [synth.picture(L, cfg, i) for i in range(n)], synth.refpics(L, cfg))


def test_gpu_444_slice_band(L, dec):
    """h264r_decode_batch_rows on 4:4:4: a band of an idc-2 slice layout equals the same rows of
    the whole picture, in all three planes."""
    cfg = synth.default_cfg(L, 4, 22, 12, chroma_format=3, num_slices=2, deblock_idc=2)
    pics = [synth.picture(L, cfg, i) for i in range(3)]
    _batch(dec, pics, synth.refpics(L, cfg), deblocks=(A.DBG_DEBLOCK_ROWS,), rows=(6, 12))


def test_gpu_444_per_picture_tables(L, dec):
    """ref_planes_stride (ABI 2) on 4:4:4: every picture reads its own DPB table, and k_derive444
    turns each into the plane's table -- picture k's slot 0 is reference k."""
    import torch
    cfg = synth.default_cfg(L, 3, 11, 9, chroma_format=3, num_refs=1)
    pics = [synth.picture(L, cfg, i) for i in range(3)]
    base = synth.refpics(L, cfg)[0]
    refs = [tuple(np.ascontiguousarray(np.roll(a, 7 * k, axis=1)) for a in base) for k in range(3)]
    dev = [[torch.from_numpy(np.concatenate([a.reshape(-1), np.zeros(64, np.uint8)])).to("cuda") for a in r] for r in refs]
    tab = np.zeros((3, 3 * A.MAX_SLOTS), np.int64)
    for k in range(3):
        for pl in range(3):
            tab[k, pl] = dev[k][pl].data_ptr()
    dtab = torch.from_numpy(tab.reshape(-1)).to("cuda")
    db = B.to_device(B.pack(pics, h264r.quant_flat()), 3, dtab.data_ptr())
    db.batch.ref_planes_stride = 3 * A.MAX_SLOTS
    dec.decode_batch(db.batch)
    dec.check()
    for k in range(3):
        want = O.decode(pics[k], [refs[k]])
        got = db.planes(k)
        for pl in range(3):
            assert _diff(got[pl], want[pl]) is None, f"picture {k} plane {pl}"


def test_gpu_444_streaming_keeps_a_reference(L, dec):
    """The streaming API (the shim's path): an I picture kept as slot 2, then a P picture
    predicting from it -- each against the oracle."""
    icfg = synth.default_cfg(L, 2, 22, 9, chroma_format=3, seed=0x444)
    pcfg = synth.default_cfg(L, 3, 22, 9, chroma_format=3, num_refs=1, seed=0x445)
    p_i = synth.picture(L, icfg, 0)
    p_p = synth.picture(L, pcfg, 0)
    for sl in p_p.slices:
        sl["ref_slot"][0][0] = 2
    got_i = dec.decode_picture(p_i, keep_slot=2)
    want_i = O.decode(p_i, [])
    for k in range(3):
        assert _diff(got_i[k], want_i[k]) is None, f"I plane {k}"
    got_p = dec.decode_picture(p_p)
    want_p = O.decode(p_p, [want_i, want_i, want_i])          # slot 2 is the one read
    for k in range(3):
        assert _diff(got_p[k], want_p[k]) is None, f"P plane {k}"


def test_gpu_444_refusals(L):
    """>8-bit stays refused; a 4:4:4 field picture is refused, not decoded wrongly."""
    import ctypes as C
    h = C.c_void_p()
    assert L.h264r_create(C.byref(h), 0, 10, 10, 3, 10) == A.EUNSUPPORTED
    d = h264r.Decoder(0, 22, 18, chroma_format=3)
    try:
        cfg = synth.default_cfg(L, 2, 22, 9, chroma_format=3, seed=0x446)
        p = synth.picture(L, cfg, 0)
        p.pic["structure"] = A.TOP_FIELD
        with pytest.raises(h264r.H264RError):
            d.decode_picture(p)
    finally:
        d.close()
