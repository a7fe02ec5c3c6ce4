"""Separate colour planes (JV, separate_colour_plane_flag) on MI355X against the reference.

Each colour plane of a JV frame is a monochrome picture with its own MBs (h264r_batch.colour_plane on
a 4:4:4 context, include/h264r.h); the fixtures are the unmodified reference's own JV decode of each
plane (tests/golden/golden.json jv_fixtures, oracle/ref_driver.cc JV mode).  The three planes of a
frame are decoded by three batches into one 4:4:4 output frame and each plane must equal the
reference's bytes.
"""
import hashlib
import json
import os
from collections import defaultdict

import numpy as np
import pytest

import _oracle as O
import h264r
from h264r import _abi as A
from h264r import batch as B
from h264r import synth

pytestmark = pytest.mark.gpu

JV = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))["jv_fixtures"]
FRAMES = defaultdict(list)
for f in JV:
    FRAMES[f["name"]].append(f)


def md5(a):
    return hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def L():
    h264r.build()
    return h264r.lib()


@pytest.fixture(scope="module")
def dec444(L):
    d = h264r.Decoder(0, 64, 36, chroma_format=3)
    yield d
    d.close()


def _decode_plane(dec, L, p, k, quant, out=None):
    host = B.pack([p], quant)
    host["chroma_format"] = 3                 # the output is the 4:4:4 frame; plane k of it is written
    db = B.to_device(host, 1, None)
    if out is not None:                       # decode into a frame shared by the three planes
        for key in ("out_y", "out_u", "out_v"):
            db.tensors[key] = out[key]
            setattr(db.batch, key, out[key].data_ptr())
    db.batch.colour_plane = k + 1
    dec.decode_batch(db.batch)
    dec.check()
    return db


@pytest.mark.parametrize("name", sorted(FRAMES))
def test_gpu_jv_frame_matches_reference(L, dec444, name):
    fxs = sorted(FRAMES[name], key=lambda f: f["colour_plane"])
    cfg = A.SynthCfg.from_dict(fxs[0]["cfg"])
    qm = fxs[0].get("qmatrix")
    quant = h264r.quant_lists(qm["m4"], qm["m8"]) if qm else h264r.quant_flat()
    r444 = synth.refpics(L, synth.default_cfg(L, 3, cfg.width_mbs, cfg.height_mbs, chroma_format=3,
                                              num_refs=cfg.num_refs, seed=cfg.seed))
    for s, (y, u, v) in enumerate(r444):
        dec444.set_ref(s, y, u, v)
    frame = None
    for fx in fxs:
        p = synth.picture(L, cfg, fx["index"])
        assert synth.input_digest(p) == fx["input_md5"]
        db = _decode_plane(dec444, L, p, fx["colour_plane"], quant, frame)
        frame = frame or {k: db.tensors[k] for k in ("out_y", "out_u", "out_v")}
    planes = db.planes(0)
    for fx in fxs:
        k = fx["colour_plane"]
        if md5(planes[k]) != fx["out_md5"]:
            want = O.decode_jv_plane(synth.picture(L, cfg, fx["index"]), k,
                                     (np.array(qm["m4"]), np.array(qm["m8"])) if qm else None)
            bad = np.argwhere(planes[k] != want)
            pytest.fail(f"plane {k}: {len(bad)} samples differ, first at {tuple(bad[0]) if len(bad) else None}")


def test_gpu_jv_refused_off_444(L):
    """colour_plane on a 4:2:0 context is H264R_EUNSUPPORTED."""
    cfg = synth.default_cfg(L, 2, 11, 9, chroma_format=A.SYNTH_CHROMA_400)
    d = h264r.Decoder(0, 11, 9)
    try:
        host = B.pack([synth.picture(L, cfg, 0)], h264r.quant_flat())
        db = B.to_device(host, 1, None)
        db.batch.colour_plane = 1
        with pytest.raises(h264r.H264RError):
            d.decode_batch(db.batch)
    finally:
        d.close()
