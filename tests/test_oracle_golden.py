"""The CPU oracle against the reference's own output bytes (tests/golden/golden.json).

golden.json was produced by tests/golden/make_golden.py from the compiled
reference decoder; every fixture is regenerated here from its seeded synth
configuration and the oracle must reproduce the reference's per-plane MD5 of
the reconstruction before deblocking and of the final deblocked picture.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import _oracle as O
from h264r import synth

_G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
GOLDEN = _G["fixtures"]
JV = _G["jv_fixtures"]


def md5(a):
    return hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("fx", GOLDEN, ids=[f"{f['name']}[{f['index']}]" for f in GOLDEN])
def test_oracle_matches_reference_fixture(fx):
    L = O.lib()
    cfg = synth.A.SynthCfg.from_dict(fx["cfg"])
    p = synth.picture(L, cfg, fx["index"])
    assert synth.input_digest(p) == fx["input_md5"], "synthetic generator drifted from the fixture"
    quant = O.quant_lists(fx["qmatrix"]["m4"], fx["qmatrix"]["m8"]) if "qmatrix" in fx else None
    rec = O.decode(p, stage="recon", quant=quant)
    assert {k: md5(rec[i]) for i, k in enumerate("YUV")} == fx["recon_md5"]
    out = O.decode(p, stage="full", quant=quant)
    assert {k: md5(out[i]) for i, k in enumerate("YUV")} == fx["out_md5"]


@pytest.mark.parametrize("fx", JV, ids=[f"{f['name']}[plane {f['colour_plane']}]" for f in JV])
def test_oracle_matches_reference_jv_plane(fx):
    """Separate colour planes (JV): the restatement (a 4:0:0 decode with plane k's lists and
    references) reproduces the reference's own JV decode of colour plane k."""
    cfg = synth.A.SynthCfg.from_dict(fx["cfg"])
    p = synth.picture(O.lib(), cfg, fx["index"])
    assert synth.input_digest(p) == fx["input_md5"], "synthetic generator drifted from the fixture"
    qm = (np.array(fx["qmatrix"]["m4"]), np.array(fx["qmatrix"]["m8"])) if "qmatrix" in fx else None
    assert md5(O.decode_jv_plane(p, fx["colour_plane"], qm)) == fx["out_md5"]


def test_fixture_coverage():
    """The fixtures exercise every feature the path claims."""
    names = {f["name"] for f in GOLDEN}
    assert sum("mbaff" in n for n in names) >= 9                           # MBAFF frames (F30)
    assert {f["colour_plane"] for f in JV} == {0, 1, 2}                   # separate colour planes (F30)
    cfgs = [f["cfg"] for f in GOLDEN]
    assert any(c["kind"] == 0 for c in cfgs) and any(c["kind"] == 1 for c in cfgs) and any(c["kind"] == 2 for c in cfgs)
    assert {0, 1, 2} <= {c["wp_mode"] for c in cfgs}
    assert {0, 1, 2} <= {c["deblock_idc"] for c in cfgs}
    assert any(c["constrained_intra"] for c in cfgs)
    assert any(c["pcm_permille"] for c in cfgs)
    assert any(c["transform8x8"] for c in cfgs) and any(not c["transform8x8"] for c in cfgs)
    assert any(c["num_slices"] > 1 for c in cfgs)
    assert any(c["filter_offset_a"] != 0 for c in cfgs)
    assert "p_1080p" in names and "intra_1080p" in names
    assert any(c.get("lossless_permille") for c in cfgs)                      # F12
    assert any(c.get("sp_slices") for c in cfgs)                              # F13 (SP)
    assert any("qmatrix" in f and f["cfg"]["kind"] == 2 for f in GOLDEN)        # scaling lists, B
    assert any(c["width_mbs"] == 240 for c in cfgs)                            # a 2160p-wide strip
    # field pictures (PAFF) of both parities, I / P / B, and one of 1080i's size
    assert {(c.get("structure", 0), c["kind"]) for c in cfgs} >= {(s, k) for s in (1, 2) for k in (0, 1, 2)}
    assert any(c.get("structure") and c["width_mbs"] == 120 and c["height_mbs"] == 34 for c in cfgs)


@pytest.mark.reference
@pytest.mark.skipif(not O.reference_available(), reason="needs /root/reference")
@pytest.mark.parametrize("cidx,over,idx", [
    (3, dict(qp_min=0, qp_max=51, mv_range_x=40, mv_range_y=40), 7),
    (4, dict(num_slices=2, deblock_idc=0, wp_mode=1, num_refs=3), 5),
    (2, dict(constrained_intra=1, pcm_permille=50, qp_min=0, qp_max=51), 9),
])
def test_oracle_vs_live_reference(cidx, over, idx):
    """Fresh seeds straight against the compiled reference (this container only)."""
    L = O.lib()
    cfg = synth.default_cfg(L, cidx, 13, 7, **over)
    p = synth.picture(L, cfg, idx)
    ref = O.run_reference(cfg, idx)
    out = O.decode(p)
    for k in range(3):
        np.testing.assert_array_equal(out[k], ref[k])
