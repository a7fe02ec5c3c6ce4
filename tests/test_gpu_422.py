"""4:2:2 pictures (chroma_format_idc 2) on the GPU path against the oracle.

A 4:2:2 MB carries 8 x 16 chroma samples per plane: eight 4x4 blocks and a 2x4 DC matrix
(transform_chroma_dc transform.cc:890-908), chroma intra prediction with the plane constants of
yCF 4 (intra_prediction.cc:871-894), chroma vectors in quarter rows (get_block_chroma
inter_prediction.cc:381-383) and four horizontal chroma edges per MB (deblock.cc:273-274).  The
library decodes the luma by the 4:2:0 launch sequence and the chroma by k_c422_inter / k_c422_intra / k_c422_db
(k_chroma422.hip, h264r_host.hip run_422).  The oracle is pinned to the compiled reference on
4:2:2 pictures by the golden fixtures (tests/golden/golden.json, the *422* cases, also run by
test_gpu_parity.py); these tests add batches under every deblocking schedule -- with 8x8
transforms too, where the chroma rows 4 / 12 of a transform-8x8 MB take the bS of 8.7.2.1
(oracle/h264r_oracle.c strength: the reference leaves it unset) -- the reconstruction alone,
per-picture DPB tables, a slice band, the streaming API keeping a picture as a reference, and
the refusals.  Bit-exact on every sample.
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
    d = h264r.Decoder(0, 240, 135, chroma_format=2)
    yield d
    d.close()


DEBLOCKS = (A.DBG_DEBLOCK_MB, A.DBG_DEBLOCK_ROWS, A.DBG_DEBLOCK_SPLIT)


def _diff(a, b):
    bad = np.argwhere(a != b)
    return None if not len(bad) else f"{len(bad)} samples differ, first at (y, x) = {tuple(bad[0])}"


def _batch(dec, pics, refs, deblocks=DEBLOCKS, rows=None, stage="full"):
    for s, (y, u, v) in enumerate(refs):
        dec.set_ref(s, y, u, v)
    want = [O.decode(p, refs, stage=stage) for p in pics]
    host = B.pack(pics, h264r.quant_flat())
    H = pics[0].cfg.height_mbs
    r0, r1 = rows if rows else (0, H)
    for db_flag in deblocks:
        db = B.to_device(host, len(pics), None)
        dec.set_debug(db_flag | (A.DBG_NO_DEBLOCK if stage == "recon" else 0))
        try:
            dec.decode_batch(db.batch, rows=rows)
            dec.check()
        finally:
            dec.set_debug(0)
        for i in range(len(pics)):
            got = db.planes(i)
            for k in range(3):
                d = _diff(got[k][r0 * 16:r1 * 16], want[i][k][r0 * 16:r1 * 16])
                assert d is None, f"{stage} deblock flag {db_flag} picture {i} plane {k}: {d}"


CASES = [
    (2, 22, 9, 3, dict(pcm_permille=30, transform8x8=0)),
    (2, 22, 9, 2, dict(constrained_intra=1)),                          # I_8x8 MBs: transform 8x8
    (3, 22, 9, 4, dict(num_refs=2)),
    (3, 22, 9, 3, dict(wp_mode=1, num_refs=3, intra_permille=250, pcm_permille=20)),
    (3, 22, 9, 3, dict(num_refs=2, transform8x8=1, intra_permille=300)),
    (4, 22, 9, 4, dict(num_refs=4)),
    (4, 22, 9, 3, dict(wp_mode=1, num_refs=4, num_slices=3, deblock_idc=2)),
    (3, 11, 9, 3, dict(qp_min=0, qp_max=20, lossless_permille=500)),
    (3, 11, 9, 2, dict(qp_min=30, qp_max=51, constrained_intra=1, intra_permille=500, mv_range_x=200, mv_range_y=120)),
    (4, 120, 17, 2, dict()),                                     # 1080p-wide
]


@pytest.mark.parametrize("cidx,W,H,n,over", CASES)
def test_gpu_422_batches(L, dec, cidx, W, H, n, over):
    cfg = synth.default_cfg(L, cidx, W, H, chroma_format=2, **over)
    _batch(dec, [synth.picture(L, cfg, i) for i in range(n)], synth.refpics(L, cfg))


@pytest.mark.parametrize("cidx,W,H,n,over", [CASES[0], CASES[3], CASES[6], CASES[7]])
def test_gpu_422_reconstruction(L, dec, cidx, W, H, n, over):
    """The chroma reconstruction alone (H264R_DBG_NO_DEBLOCK) against the oracle's pre-deblocking planes."""
    cfg = synth.default_cfg(L, cidx, W, H, chroma_format=2, **over)
    _batch(dec, [synth.picture(L, cfg, i) for i in range(n)], synth.refpics(L, cfg), deblocks=(0,), stage="recon")


def test_gpu_422_slice_band(L, dec):
    """h264r_decode_batch_rows on 4:2:2: a band of an idc-2 slice layout equals the same rows of
    the whole picture, in all three planes (chroma rows 16 per MB row)."""
    cfg = synth.default_cfg(L, 4, 22, 12, chroma_format=2, num_slices=2, deblock_idc=2)
    pics = [synth.picture(L, cfg, i) for i in range(3)]
    _batch(dec, pics, synth.refpics(L, cfg), deblocks=(A.DBG_DEBLOCK_ROWS,), rows=(6, 12))


def test_gpu_422_per_picture_tables(L, dec):
    """ref_planes_stride (ABI 2) on 4:2:2: every picture reads its own DPB table -- its luma
    through k_derive444's plane-0 table, its chroma through the table itself (k_c422_inter)."""
    import torch
    cfg = synth.default_cfg(L, 3, 11, 9, chroma_format=2, num_refs=1)
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


def test_gpu_422_streaming_keeps_a_reference(L, dec):
    """The streaming API (the shim's path): an I picture kept as slot 2, then a P picture
    predicting from it -- each against the oracle."""
    icfg = synth.default_cfg(L, 2, 22, 9, chroma_format=2, seed=0x422)
    pcfg = synth.default_cfg(L, 3, 22, 9, chroma_format=2, num_refs=1, seed=0x423)
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


def test_gpu_422_refusals(L):
    """Bit depths above 8 stay refused; a 4:2:2 field picture and a 4:2:2 SP slice (Extended
    profile is 4:2:0) are refused, not decoded wrongly."""
    import ctypes as C
    h = C.c_void_p()
    assert L.h264r_create(C.byref(h), 0, 10, 10, 5, 8) == A.EUNSUPPORTED
    assert L.h264r_create(C.byref(h), 0, 10, 10, 2, 10) == A.EUNSUPPORTED
    d = h264r.Decoder(0, 22, 18, chroma_format=2)
    try:
        cfg = synth.default_cfg(L, 2, 22, 9, chroma_format=2, seed=0x424)
        p = synth.picture(L, cfg, 0)
        p.pic["structure"] = A.TOP_FIELD
        with pytest.raises(h264r.H264RError):
            d.decode_picture(p)
        cfg = synth.default_cfg(L, 3, 22, 9, chroma_format=2, num_refs=1, seed=0x425)
        p = synth.picture(L, cfg, 0)
        p.slices["slice_type"] = A.SLICE_SP
        with pytest.raises(h264r.H264RError):
            d.decode_picture(p, synth.refpics(L, cfg))
    finally:
        d.close()
