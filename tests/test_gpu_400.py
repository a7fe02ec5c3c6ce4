"""4:0:0 pictures (chroma_format_idc 0, monochrome) on the GPU path against the oracle.

A 4:0:0 picture has no chroma at all: no chroma prediction, residual, PCM samples or deblocking
(decoder.cc:199, deblock.cc:498,522; picture.cc:34 allocates no chroma planes).  The library
decodes its luma by the 4:2:0 launch sequence (h264r_host.hip run_422: k_derive444 plane 0, the
chroma of that pass into scratch) and writes nothing else.  The oracle is pinned to the compiled
reference on 4:0:0 pictures by the golden fixtures (the *400* cases, also run by
test_gpu_parity.py); these tests add batches under every deblocking schedule, the streaming API
keeping a picture as a reference, and the refusals.  Bit-exact on every luma sample.
"""
import numpy as np
import pytest

import _oracle as O
import h264r
from h264r import _abi as A
from h264r import batch as B
from h264r import synth

pytestmark = pytest.mark.gpu

C400 = A.SYNTH_CHROMA_400


@pytest.fixture(scope="module")
def L():
    h264r.build()
    return h264r.lib()


@pytest.fixture(scope="module")
def dec(L):
    d = h264r.Decoder(0, 240, 135, chroma_format=0)
    yield d
    d.close()


@pytest.mark.parametrize("cidx,W,H,n,over", [
    (2, 22, 9, 3, dict(pcm_permille=30)),
    (3, 22, 9, 3, dict(wp_mode=1, num_refs=3, intra_permille=250, pcm_permille=20, constrained_intra=1)),
    (4, 22, 9, 3, dict(num_refs=4, num_slices=3, deblock_idc=2)),
    (3, 11, 9, 3, dict(qp_min=0, qp_max=20, lossless_permille=500)),
    (4, 120, 17, 2, dict()),
])
def test_gpu_400_batches(L, dec, cidx, W, H, n, over):
    cfg = synth.default_cfg(L, cidx, W, H, chroma_format=C400, **over)
    pics = [synth.picture(L, cfg, i) for i in range(n)]
    refs = synth.refpics(L, cfg)
    for s, (y, u, v) in enumerate(refs):
        dec.set_ref(s, y, u, v)
    want = [O.decode(p, refs) for p in pics]
    host = B.pack(pics, h264r.quant_flat())
    for flag in (A.DBG_DEBLOCK_MB, A.DBG_DEBLOCK_ROWS, A.DBG_DEBLOCK_SPLIT):
        db = B.to_device(host, n, None)
        dec.set_debug(flag)
        try:
            dec.decode_batch(db.batch)
            dec.check()
        finally:
            dec.set_debug(0)
        for i in range(n):
            got = db.planes(i)[0]
            bad = np.argwhere(got != want[i][0])
            assert not len(bad), f"deblock flag {flag} picture {i}: {len(bad)} samples differ, first {tuple(bad[0])}"


def test_gpu_400_streaming_keeps_a_reference(L, dec):
    icfg = synth.default_cfg(L, 2, 22, 9, chroma_format=C400, seed=0x400)
    pcfg = synth.default_cfg(L, 3, 22, 9, chroma_format=C400, num_refs=1, seed=0x401)
    p_i, p_p = synth.picture(L, icfg, 0), synth.picture(L, pcfg, 0)
    for sl in p_p.slices:
        sl["ref_slot"][0][0] = 3
    got_i = dec.decode_picture(p_i, keep_slot=3)
    want_i = O.decode(p_i, [])
    assert np.array_equal(got_i[0], want_i[0])
    got_p = dec.decode_picture(p_p)
    want_p = O.decode(p_p, [want_i] * 4)
    assert np.array_equal(got_p[0], want_p[0])


def test_gpu_400_refusals(L):
    """A 4:0:0 field picture and SP slices are refused, not decoded wrongly."""
    d = h264r.Decoder(0, 22, 18, chroma_format=0)
    try:
        cfg = synth.default_cfg(L, 2, 22, 9, chroma_format=C400, seed=0x402)
        p = synth.picture(L, cfg, 0)
        p.pic["structure"] = A.TOP_FIELD
        with pytest.raises(h264r.H264RError):
            d.decode_picture(p)
        cfg = synth.default_cfg(L, 3, 22, 9, chroma_format=C400, num_refs=1, seed=0x403)
        p = synth.picture(L, cfg, 0)
        p.slices["slice_type"] = A.SLICE_SP
        with pytest.raises(h264r.H264RError):
            d.decode_picture(p, synth.refpics(L, cfg))
    finally:
        d.close()
