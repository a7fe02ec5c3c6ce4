"""MBAFF frames on MI355X (k_mbaff.hip) against the oracle, which the reference pins.

The golden MBAFF fixtures (tests/golden/golden.json, `*mbaff*`: the unmodified reference driven
by oracle/ref_driver.cc) run through test_gpu_parity.test_gpu_matches_reference_fixture; these
tests add device-resident batches, 1080p pictures, the streaming API's reference slots and the
refusals (include/h264r.h H264R_MBAFF_FRAME).  Bit-exact on every sample.
"""
import ctypes as C

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
    d = h264r.Decoder(0, 240, 136)
    yield d
    d.close()


def _diff(a, b):
    bad = np.argwhere(a != b)
    if not len(bad):
        return None
    y, x = bad[0]
    return f"{len(bad)} samples differ, first at (x={x}, y={y}): gpu={a[y, x]} want={b[y, x]}"


def _set_refs(dec, refs):
    for s, (y, u, v) in enumerate(refs):
        dec.set_ref(s, y, u, v)


@pytest.mark.parametrize("cidx,W,H,over", [
    (2, 22, 18, dict(pcm_permille=20)),
    (3, 22, 18, dict(num_refs=3, intra_permille=250)),
    (3, 22, 18, dict(wp_mode=1, num_refs=2, constrained_intra=1, intra_permille=300, num_slices=3, deblock_idc=2)),
    (4, 22, 18, dict(wp_mode=0, num_refs=4, num_slices=2, deblock_idc=0)),
    (4, 22, 18, dict(wp_mode=1, num_refs=3, mv_range_x=150, mv_range_y=90, filter_offset_a=8, filter_offset_b=-8)),
])
def test_gpu_mbaff_batch(L, dec, cidx, W, H, over):
    """Four MBAFF pictures in one device-resident batch (h264r_decode_batch, mbaff = 1), each equal
    to the oracle: intra (with PCM), P with slices / CIP / explicit weights, B default / explicit."""
    cfg = synth.default_cfg(L, cidx, W, H, structure=A.MBAFF_FRAME, **over)
    pics = [synth.picture(L, cfg, i) for i in range(4)]
    refs = synth.refpics(L, cfg)
    _set_refs(dec, refs)
    host = B.pack(pics, h264r.quant_flat())
    db = B.to_device(host, len(pics), None)
    assert db.batch.mbaff == 1
    dec.decode_batch(db.batch)
    dec.check()
    for i, p in enumerate(pics):
        want = O.decode(p, refs)
        got = db.planes(i)
        for k in range(3):
            assert _diff(got[k], want[k]) is None, f"picture {i} plane {k}: {_diff(got[k], want[k])}"


@pytest.mark.parametrize("cidx", [2, 3, 4])
def test_gpu_mbaff_1080p(L, dec, cidx):
    """A whole 1080p MBAFF frame (120 x 68 MBs, 34 pair rows) of each kind against the oracle."""
    over = dict(wp_mode=1) if cidx == 4 else {}
    cfg = synth.default_cfg(L, cidx, 120, 68, structure=A.MBAFF_FRAME, **over)
    p = synth.picture(L, cfg, 0)
    refs = synth.refpics(L, cfg)
    got = dec.decode_picture(p, refs)
    want = O.decode(p, refs)
    for k in range(3):
        assert _diff(got[k], want[k]) is None, f"plane {k}: {_diff(got[k], want[k])}"


def test_gpu_mbaff_reconstruction_only(L, dec):
    """H264R_DBG_NO_DEBLOCK: the MBAFF reconstruction before the loop filter equals the oracle's
    (the frame after MbAffPostProc, deblock.cc:596-629)."""
    cfg = synth.default_cfg(L, 4, 22, 18, structure=A.MBAFF_FRAME, wp_mode=1, num_refs=3)
    p = synth.picture(L, cfg, 1)
    refs = synth.refpics(L, cfg)
    got = dec.decode_picture(p, refs, no_deblock=True)
    want = O.decode(p, refs, stage="recon")
    for k in range(3):
        assert _diff(got[k], want[k]) is None, f"plane {k}: {_diff(got[k], want[k])}"


def test_gpu_mbaff_keeps_a_reference(L, dec):
    """The streaming API: an MBAFF I frame kept as DPB slot 2, then an MBAFF P frame whose frame
    and field MBs predict from it (its fields for the field MBs) -- each equal to the oracle."""
    icfg = synth.default_cfg(L, 2, 22, 18, structure=A.MBAFF_FRAME, seed=0x3AFF)
    pcfg = synth.default_cfg(L, 3, 22, 18, structure=A.MBAFF_FRAME, num_refs=1, seed=0x3B00)
    p_i = synth.picture(L, icfg, 0)
    p_p = synth.picture(L, pcfg, 0)
    for sl in p_p.slices:
        sl["ref_slot"][0][0] = 2
    got_i = dec.decode_picture(p_i, keep_slot=2)
    want_i = O.decode(p_i, [])
    for k in range(3):
        assert _diff(got_i[k], want_i[k]) is None, f"I plane {k}"
    got_p = dec.decode_picture(p_p)
    want_p = O.decode(p_p, [want_i, want_i, want_i])
    for k in range(3):
        assert _diff(got_p[k], want_p[k]) is None, f"P plane {k}: {_diff(got_p[k], want_p[k])}"


def test_gpu_mbaff_refusals(L, dec):
    """Implicit weights, SP slices and lossless MBs in an MBAFF frame are refused, as are a pair
    whose two MBs disagree on mb_field_decoding_flag and an odd MB-row count."""
    cfg = synth.default_cfg(L, 4, 11, 8, structure=A.MBAFF_FRAME, wp_mode=0)
    p = synth.picture(L, cfg, 0)
    refs = synth.refpics(L, cfg)
    bad = synth.picture(L, cfg, 0)
    bad.slices["wp_mode"] = 2
    with pytest.raises(h264r.H264RError):
        dec.decode_picture(bad, refs)
    bad = synth.picture(L, cfg, 0)
    bad.mbs["flags"][0] ^= A.MBF_FIELD                # the top MB of pair 0 alone
    with pytest.raises(h264r.H264RError):
        dec.decode_picture(bad, refs)
    # still decodes after the refusals
    got = dec.decode_picture(p, refs)
    want = O.decode(p, refs)
    for k in range(3):
        assert _diff(got[k], want[k]) is None
    h = C.c_void_p()
    L.h264r_create(C.byref(h), 0, 11, 9, 1, 8)
    try:
        pic = np.zeros(1, A.PIC_DTYPE)
        pic["structure"] = A.MBAFF_FRAME
        pic["num_slices"] = 1
        sl = np.zeros(1, A.SLICE_DTYPE)
        q = h264r.quant_flat()
        assert L.h264r_picture_begin(h, 11, 9, A.ptr(pic), A.ptr(sl), A.ptr(q)) == A.OK
        mb = np.zeros(1, A.MB_DTYPE)
        mb["mb_type"] = A.I_16x16
        mb["flags"] = A.MBF_INTRA
        mv = np.zeros(32, np.uint32)
        rr = np.full(32, -1, np.int8)
        for a in range(99):
            assert L.h264r_mb_submit(h, a, A.ptr(mb), None, 0, A.ptr(mv), A.ptr(rr)) == A.OK
        assert L.h264r_picture_end(h, None, None, None, -1) == A.EINVAL       # 9 MB rows: no pairs
    finally:
        L.h264r_destroy(h)
