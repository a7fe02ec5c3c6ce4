"""Field pictures (PAFF) on the GPU path (lib/libh264r.so on gfx950) against the oracle.

A field picture is reconstructed and deblocked as a picture of half the frame's MB rows whose
references are fields of the DPB's frames (include/h264r.h H264R_TOP_FIELD): every second row
of a slot, the chroma parity offset of get_block_chroma (inter_prediction.cc:352-355), field
deblocking rules (mvlimit 2, bS 3 across horizontal MB edges, deblock.cc:86-189).  The oracle
is pinned to the compiled reference on field pictures by the golden fixtures
(tests/golden/golden.json, the *field_* cases, also run by test_gpu_parity.py); these tests add
batches, both parities in one launch, the slice-band form and the streaming API's field pairs
sharing one DPB slot.  Bit-exact on every sample.
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
    d = h264r.Decoder(0, 240, 135)
    yield d
    d.close()


DEBLOCKS = (A.DBG_DEBLOCK_MB, A.DBG_DEBLOCK_ROWS, A.DBG_DEBLOCK_SPLIT)


def _diff(a, b):
    bad = np.argwhere(a != b)
    return None if not len(bad) else f"{len(bad)} samples differ, first at (y, x) = {tuple(bad[0])}"


def _batch(L, dec, pics, refs, deblocks=DEBLOCKS, rows=None):
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
                m = 16 if k == 0 else 8
                d = _diff(got[k][r0 * m:r1 * m], want[i][k][r0 * m:r1 * m])
                assert d is None, f"deblock flag {db_flag} picture {i} plane {k}: {d}"


@pytest.mark.parametrize("cidx,W,H,n,over", [
    (3, 22, 9, 6, dict(structure=1, num_refs=4)),
    (3, 22, 9, 5, dict(structure=2, num_refs=3, pcm_permille=30, intra_permille=250)),
    (4, 22, 9, 4, dict(structure=1, num_refs=4, num_slices=3, deblock_idc=2)),
    (4, 22, 9, 4, dict(structure=2, wp_mode=1, num_refs=6, mv_range_x=200, mv_range_y=100)),
    (2, 22, 9, 3, dict(structure=1, pcm_permille=20)),
    (3, 22, 9, 4, dict(structure=2, sp_slices=1, num_refs=2)),
    (4, 11, 4, 4, dict(structure=1, qp_min=0, qp_max=20, lossless_permille=500)),
    (3, 120, 34, 4, dict(structure=1)),                  # 1080i: a field of a 1080p frame
    (4, 120, 34, 3, dict(structure=2)),
])
def test_gpu_field_batches(L, dec, cidx, W, H, n, over):
    cfg = synth.default_cfg(L, cidx, W, H, **over)
    _batch(L, dec, [synth.picture(L, cfg, i) for i in range(n)], synth.refpics(L, cfg))


def test_gpu_field_batch_both_parities(L, dec):
    """Top and bottom fields (and their opposite-parity chroma offsets) in one launch."""
    top = synth.default_cfg(L, 4, 22, 9, structure=1, num_refs=4, seed=0x71)
    bot = synth.default_cfg(L, 4, 22, 9, structure=2, num_refs=4, seed=0x72)
    pics = [synth.picture(L, top if i % 2 == 0 else bot, i) for i in range(6)]
    _batch(L, dec, pics, synth.refpics(L, top))


def test_gpu_field_slice_band(L, dec):
    """The slice-sharded form (h264r_decode_batch_rows) on field pictures: a band of an idc-2
    slice layout equals the same rows of the whole field."""
    cfg = synth.default_cfg(L, 4, 120, 34, structure=2, num_slices=2, deblock_idc=2)
    pics = [synth.picture(L, cfg, i) for i in range(3)]
    rows = (17, 34)
    _batch(L, dec, pics, synth.refpics(L, cfg), deblocks=(A.DBG_DEBLOCK_ROWS,), rows=rows)


def _interleave(top, bot):
    out = []
    for t, b in zip(top, bot):
        f = np.empty((2 * t.shape[0], t.shape[1]), np.uint8)
        f[0::2], f[1::2] = t, b
        out.append(f)
    return tuple(out)


def test_gpu_field_pair_shares_a_slot(L, dec):
    """The streaming API (the shim's path): an I top field kept as slot 5, the bottom field
    predicting from it (its complementary field, slot 5's top rows) and from slot 0's fields,
    kept into slot 5's bottom rows, then a frame picture predicting from the frame the two
    fields make up (dpb_combine_field_yuv picture.cc:578-622) -- each against the oracle."""
    W, FH = 22, 18
    icfg = synth.default_cfg(L, 2, W, FH // 2, structure=1, seed=0x81)
    pcfg = synth.default_cfg(L, 3, W, FH // 2, structure=2, num_refs=3, seed=0x82)
    fcfg = synth.default_cfg(L, 3, W, FH, num_refs=2, seed=0x83, intra_permille=50)
    frame0 = synth.refpics(L, pcfg)[0]
    grey = tuple(np.full_like(a, 128) for a in frame0)

    p_top = synth.picture(L, icfg, 0)
    p_bot = synth.picture(L, pcfg, 0)
    # list 0 of the bottom field: the top field of slot 5 first (8.2.4.2.5 puts the same
    # parity first, but any order is a valid list), then slot 0's fields
    for sl in p_bot.slices:
        sl["ref_slot"][0][:3] = [5, 0 | A.REF_BOTTOM, 0]
    p_frm = synth.picture(L, fcfg, 0)
    for sl in p_frm.slices:
        sl["ref_slot"][0][:2] = [5, 0]

    dec.set_ref(0, *frame0)
    got_top = dec.decode_picture(p_top, keep_slot=5)
    want_top = O.decode(p_top, [frame0])
    for k in range(3):
        assert _diff(got_top[k], want_top[k]) is None, f"top field plane {k}"
    # the bottom rows are not read by the bottom field (any content)
    slot5 = _interleave(want_top, tuple(np.full_like(a, 128) for a in want_top))
    refs = [frame0] + [grey] * 4 + [slot5]
    got_bot = dec.decode_picture(p_bot, keep_slot=5)
    want_bot = O.decode(p_bot, refs)
    for k in range(3):
        assert _diff(got_bot[k], want_bot[k]) is None, f"bottom field plane {k}"
    refs[5] = _interleave(want_top, want_bot)
    got_frm = dec.decode_picture(p_frm)
    want_frm = O.decode(p_frm, refs)
    for k in range(3):
        assert _diff(got_frm[k], want_frm[k]) is None, f"frame plane {k}"


def test_gpu_field_streaming_errors(L, dec):
    """A field picture whose list names a slot of the wrong size, or a parity bit in a frame
    picture's list, is refused, not predicted from the wrong rows."""
    cfg = synth.default_cfg(L, 3, 11, 4, structure=1, num_refs=2, seed=0x91)
    p = synth.picture(L, cfg, 0)
    y, u, v = synth.refpics(L, cfg)[0]
    dec.set_ref(0, y[:64], u[:32], v[:32])               # a frame of the FIELD's height: wrong size
    with pytest.raises(h264r.H264RError):
        dec.decode_picture(p)
    fcfg = synth.default_cfg(L, 3, 11, 8, num_refs=1, seed=0x92)
    q = synth.picture(L, fcfg, 0)
    dec.set_ref(0, y, u, v)
    for sl in q.slices:
        sl["ref_slot"][0][0] = 0 | A.REF_BOTTOM
    with pytest.raises(h264r.H264RError):
        dec.decode_picture(q)
