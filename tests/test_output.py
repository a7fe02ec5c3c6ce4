"""The output/compare step (h264r.output): cropping YUV writer and per-frame MD5 compare.

Follows write_out_picture / img2buf (src/codec/h264/framebuf/output.cc:61-227) and
the harness's digest_by_frames / compare (script/test/model/__init__.py:119-183).
The per-plane bytes are pinned by golden.json's reference out_md5 digests; the
crop arithmetic by a per-sample restatement of img2buf_byte below.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import _oracle as O
from h264r import output as OUT
from h264r import synth

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))["fixtures"]


def img2buf_loop(img, size_x, size_y, cl, cr, ct, cb, stride):
    """output.cc img2buf_byte, one sample at a time (test restatement)."""
    buf = bytearray(stride * (size_y - ct - cb))
    for j in range(ct, size_y - cb):
        for i in range(cl, size_x - cr):
            buf[(j - ct) * stride + (i - cl)] = int(img[j, i])
    return bytes(buf)


def test_geometry_1080p():
    crop = OUT.Crop.for_height(120, 68, 1920, 1080)
    assert crop == OUT.Crop(bottom=4)
    g = OUT.geometry(120, 68, crop)
    assert g.luma == (0, 0, 1920, 1080) and g.chroma == (0, 0, 960, 540)
    assert g.frame_bytes == 1920 * 1080 * 3 // 2


def test_geometry_field_and_errors():
    # frame_mbs_only_flag = 0 doubles the vertical crop units (output.cc:152-153)
    g = OUT.geometry(11, 10, OUT.Crop(left=1, right=2, top=1, bottom=1, frame_mbs_only=0))
    assert g.luma == (2, 4, 176 - 6, 160 - 8) and g.chroma == (1, 2, 88 - 3, 80 - 4)
    with pytest.raises(ValueError):
        OUT.geometry(2, 2, OUT.Crop(left=8, right=8))
    with pytest.raises(ValueError):
        OUT.Crop.for_height(120, 68, 1920, 1089)


@pytest.mark.parametrize("crop", [OUT.Crop(), OUT.Crop(left=1, right=3, top=2, bottom=1)])
def test_frame_bytes_match_img2buf(crop):
    rng = np.random.default_rng(7)
    W, H = 5, 3
    y = rng.integers(0, 256, (16 * H, 16 * W), dtype=np.uint8)
    u = rng.integers(0, 256, (8 * H, 8 * W), dtype=np.uint8)
    v = rng.integers(0, 256, (8 * H, 8 * W), dtype=np.uint8)
    g = OUT.geometry(W, H, crop)
    lc, rc, tc, bc = crop.left, crop.right, crop.top, crop.bottom
    want = (img2buf_loop(y, 16 * W, 16 * H, 2 * lc, 2 * rc, 2 * tc, 2 * bc, g.luma[2])
            + img2buf_loop(u, 8 * W, 8 * H, lc, rc, tc, bc, g.chroma[2])
            + img2buf_loop(v, 8 * W, 8 * H, lc, rc, tc, bc, g.chroma[2]))
    assert OUT.frame_bytes(y, u, v, g) == want


def test_frame_bytes_rejects_bad_planes():
    g = OUT.geometry(2, 2)
    y = np.zeros((32, 32), np.uint8)
    c = np.zeros((16, 16), np.uint8)
    with pytest.raises(ValueError):
        OUT.frame_bytes(y[:16], c, c, g)
    with pytest.raises(ValueError):
        OUT.frame_bytes(y.astype(np.uint16), c, c, g)


def test_digest_and_compare_protocol(tmp_path):
    frames = [bytes([i]) * 24 for i in range(3)]
    data = b"".join(frames)
    lines = OUT.digest_by_frames(data, 3)
    assert lines == [hashlib.md5(f).hexdigest() for f in frames]
    md5file = tmp_path / "x.yuv.md5"
    OUT.write_digests(md5file, [l.upper() for l in lines])        # the list is compared lower-case
    yuv = tmp_path / "x.yuv"
    yuv.write_bytes(data)
    assert OUT.compare_yuv(yuv, md5file, "x") == lines
    # a remainder becomes one more chunk: the frame count differs (model/__init__.py:139-147,166-167)
    with pytest.raises(OUT.CompareError, match="decoded frames is different"):
        OUT.compare(OUT.digest_by_frames(data + b"\0", 3), lines, "x")
    bad = bytearray(data)
    bad[30] ^= 1
    with pytest.raises(OUT.CompareError, match="mismatch 1 x"):
        OUT.compare(OUT.digest_by_frames(bytes(bad), 3), lines, "x")
    with pytest.raises(ValueError):
        OUT.digest_by_frames(data, 0)


def test_writer_over_oracle_sequence(tmp_path):
    """A short sequence decoded by the oracle, written uncropped: every frame's bytes are
    the reference's Y||Cb||Cr (golden out_md5 per plane), and the compare passes."""
    fxs = [f for f in GOLDEN if f["cfg"]["width_mbs"] == 11 and f["cfg"]["height_mbs"] == 9][:3]
    assert fxs
    L = O.lib()
    path = tmp_path / "seq.yuv"
    want = []
    with OUT.YuvWriter(path, 11, 9) as w:
        for fx in fxs:
            p = synth.picture(L, synth.A.SynthCfg.from_dict(fx["cfg"]), fx["index"])
            y, u, v = O.decode(p)
            for k, pl in zip("YUV", (y, u, v)):
                assert hashlib.md5(np.ascontiguousarray(pl).tobytes()).hexdigest() == fx["out_md5"][k]
            want.append(hashlib.md5(y.tobytes() + u.tobytes() + v.tobytes()).hexdigest())
            w.write(y, u, v)
    assert w.frames == len(fxs)
    OUT.write_digests(tmp_path / "seq.yuv.md5", want)
    assert OUT.compare_yuv(path, tmp_path / "seq.yuv.md5", "seq") == want
