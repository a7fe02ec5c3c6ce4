"""Stream-level parity.

Streams written by the repo's own bitstream writer are decoded
  * by the UNMODIFIED reference decoder (golden per-frame MD5s, tests/golden/streams.json),
  * by the reference's parser + the drop-in Decoder shim (shim/decoder_h264r.cc) over the
    CPU oracle -- this container only, where the reference builds,
  * on MI355X: the MB records the shim handed to the C ABI (captured fixtures) replayed
    through libh264r.so, and, when the box has it, the reference parser + shim linked
    against libh264r.so decoding the stream end to end,
and every decode must reproduce the reference's per-frame MD5s (the reference harness's
compare protocol, script/test/model/__init__.py:119-183).
"""
import ctypes as C
import json
import sys
import hashlib
import os
import subprocess

import numpy as np
import pytest

import _oracle as O
import h264_writer as Wr
import streams as S
from h264r import _abi as A
from h264r import output as OUT

GOLD = S.golden()["streams"]
NAMES = list(S.STREAMS)
REF_BIN = os.path.join(S.ROOT, "oracle", "_ref")


def _replay(pics, decode_picture):
    """Decode captured pictures in decoding order, keeping each reference picture in the
    DPB slot the shim gave it; returns the output frames in output order (POC), field
    pairs interleaved into their frames."""
    return S.output_frames(pics, [decode_picture(p) for p in pics])


def test_stream_set_matches_writer_and_golden_table():
    assert set(GOLD) == set(S.STREAMS)
    for name, cfg in S.STREAMS.items():
        assert GOLD[name]["cfg"] == {k: list(v) if isinstance(v, tuple) else v for k, v in cfg.items()}
        assert len(GOLD[name]["frame_md5"]) == cfg["frames"]


@pytest.mark.parametrize("name", NAMES)
def test_writer_reproduces_committed_stream(name):
    """The committed bitstreams are exactly what the writer produces (seeded)."""
    data = Wr.Encoder(Wr.StreamCfg(**S.STREAMS[name])).stream()
    assert data == open(S.stream_path(name), "rb").read()


def test_captures_cover_the_path():
    """The captured MB records exercise every reconstruction function the streams can
    carry: all P partitions and P_Skip, I_4x4 / I_8x8 / I_16x16 / I_PCM, both transform
    sizes, every CBP class, explicit WP, deblocking idc 0/1/2 with offsets, multi-slice
    pictures, scaling lists (non-flat quantisation tables)."""
    types, t8, wp, idc, offs, multi, nonflat, chroma = set(), False, False, set(), False, False, False, set()
    stypes, bwp, l1, t8b = set(), set(), False, False
    flat = O.quant_flat()
    for name in NAMES:
        for p in S.load_capture(S.capture_path(name)):
            m = p["mbs"]
            types |= set(int(t) for t in np.unique(m["mb_type"]))
            t8 |= bool((m["flags"] & A.MBF_T8x8).any())
            chroma |= set(int(c) for c in np.unique(m["cbp"] >> 4))
            sl = p["slices"]
            stypes |= set(int(v) for v in sl["slice_type"])
            if (sl["slice_type"] == A.SLICE_B).any():
                bwp |= set(int(v) for v in sl["wp_mode"])
                l1 |= bool((p["ref_idx"][1] >= 0).any())
                t8b |= bool((m["flags"] & A.MBF_T8x8).any())
            wp |= bool((sl["wp_mode"] == 1).any())
            idc |= set(int(v) for v in sl["deblock_idc"])
            offs |= bool((sl["filter_offset_a"] != 0).any() or (sl["filter_offset_b"] != 0).any())
            multi |= len(sl) > 1
            nonflat |= p["quant"].tobytes() != flat.tobytes()
    assert {A.P_SKIP, A.P_16x16, A.P_16x8, A.P_8x16, A.P_8x8, A.I_4x4, A.I_8x8, A.I_16x16, A.I_PCM} <= types
    assert t8 and wp and idc == {0, 1, 2} and offs and multi and nonflat and chroma == {0, 1, 2}
    # B slices with list-1 prediction under every bi-prediction weighting, 8x8 transforms in B
    assert {A.SLICE_P, A.SLICE_B, A.SLICE_I, A.SLICE_SP} <= stypes and bwp == {0, 1, 2} and l1 and t8b


@pytest.mark.parametrize("name", NAMES)
def test_oracle_replay_of_captures_matches_reference(name):
    """The CPU oracle (oracle/h264r_oracle.c) decoding the captured boundary arrays
    reproduces the unmodified reference's per-frame MD5s: pins the oracle on parsed
    streams, runs anywhere (no reference needed)."""
    cfg = S.STREAMS[name]
    pics = S.load_capture(S.capture_path(name))
    L = O.lib()
    slots = {}

    def dec(p):
        W, H = p["W"], p["H"]
        out = O.new_planes(W, H, p["chroma_format"])
        fld = S.structure(p) in (A.TOP_FIELD, A.BOTTOM_FIELD)
        o = O.OraclePicture()
        o.width_mbs, o.height_mbs = W, H
        o.chroma_format = p["chroma_format"]
        o.mbs, o.levels = A.ptr(p["mbs"]).value, A.ptr(p["levels"]).value
        o.mv, o.ref_idx = A.ptr(p["mv"]).value, A.ptr(p["ref_idx"]).value
        o.slices, o.pic, o.quant = A.ptr(p["slices"]).value, A.ptr(p["pic"]).value, A.ptr(p["quant"]).value
        for s, planes in slots.items():
            for k in range(3):
                o.ref_planes[s][k] = A.ptr(planes[k]).value
        for k in range(3):
            o.out[k] = A.ptr(out[k]).value
        assert L.oracle_decode_picture(C.byref(o)) == 0
        if p["keep"] >= 0 and not fld:
            slots[p["keep"]] = out
        elif p["keep"] >= 0:
            # a field into its parity's rows of the slot's frame (include/h264r.h)
            fr = slots.get(p["keep"])
            if fr is None or fr[0].shape != (32 * H, 16 * W):
                fr = O.new_planes(W, 2 * H)
            par = 1 if S.structure(p) == A.BOTTOM_FIELD else 0
            for k in range(3):
                fr[k][par::2] = out[k]
            slots[p["keep"]] = fr
        return out
    outs = _replay(pics, dec)
    assert S.frame_md5s(outs, cfg) == GOLD[name]["frame_md5"]


@pytest.mark.skipif(not O.reference_available(), reason="needs /root/reference (this container only)")
@pytest.mark.parametrize("name", NAMES)
def test_reference_and_shim_reproduce_golden(name, tmp_path):
    """In this container: the unmodified reference and the reference parser + drop-in
    shim (over the CPU oracle) both decode the committed stream to the golden MD5s."""
    O.build_ref()
    cfg = S.STREAMS[name]
    for binary in ("ldecod", "ldecod_shim"):
        out = tmp_path / f"{binary}.yuv"
        r = subprocess.run([os.path.join(REF_BIN, binary), "-i", S.stream_path(name), "-o", str(out)],
                           capture_output=True, text=True, timeout=600, cwd=tmp_path)
        assert r.returncode == 0, r.stdout[-800:] + r.stderr[-800:]
        assert OUT.digest_by_frames(str(out), cfg["frames"]) == GOLD[name]["frame_md5"], binary


# ---------------------------------------------------------------------------- MI355X
@pytest.mark.gpu
@pytest.mark.parametrize("flag", [A.DBG_DEBLOCK_MB, A.DBG_DEBLOCK_ROWS], ids=["deblock_mb", "deblock_rows"])
@pytest.mark.parametrize("name", NAMES)
def test_gpu_replay_of_captures_matches_reference(name, flag):
    """The MB records the reference parser handed the shim, replayed through the C ABI
    of libh264r.so on MI355X (streaming API, each reference picture kept on the device
    in the shim's DPB slot), reproduce the reference's per-frame MD5s bit for bit --
    under both deblocking schedules."""
    import h264r
    cfg = S.STREAMS[name]
    pics = S.load_capture(S.capture_path(name))
    W, H = cfg["width_mbs"], cfg["height_mbs"]
    with h264r.Decoder(0, W, H, chroma_format=cfg.get("chroma_format", 1)) as dec:
        dec.set_debug(flag)
        def run(p):
            dec.assign_quant_params(p["quant"])
            dec.init(p["W"], p["H"], p["pic"], p["slices"])           # a field: half the frame's rows
            for a, rec, lv, mv, ri in S.iter_mbs(p):
                dec.decode(a, rec, lv, mv, ri)
            return dec.deblock_filter(p["keep"])
        outs = _replay(pics, run)
    got = S.frame_md5s(outs, cfg)
    if got != GOLD[name]["frame_md5"]:
        bad = [i for i, (a, b) in enumerate(zip(got, GOLD[name]["frame_md5"])) if a != b]
        planes = {i: [hashlib.md5(x.tobytes()).hexdigest() == m for x, m in zip(outs[i], pics[i]["plane_md5"])]
                  for i in bad}
        pytest.fail(f"{name}: frames {bad} differ from the reference (Y/Cb/Cr equal to the oracle: {planes})")


CABAC_TRACED = [n for n, c in S.STREAMS.items() if c.get("cabac") and c["width_mbs"] * c["height_mbs"] <= 400]


@pytest.mark.skipif(not O.reference_available(), reason="needs /root/reference (this container only)")
@pytest.mark.parametrize("name", CABAC_TRACED)
def test_reference_parser_reads_what_the_cabac_writer_wrote(name):
    """Every syntax element the reference parser decodes from a CABAC stream (mb_skip_flag,
    mb_type, sub_mb_type, transform_size_8x8_flag, intra modes, ref_idx, mvd, CBP,
    mb_qp_delta and every coefficient it pushes through Decoder::coeff_*; traced by
    oracle/_ref/ldecod_trace) is the one the writer meant -- the MD5 agreement above could
    otherwise hide a stream both decoders misread alike."""
    O.build_ref()
    r = subprocess.run([sys.executable, os.path.join(S.ROOT, "tools", "cabac_trace_diff.py"),
                        json.dumps(S.STREAMS[name])], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "syntax elements agree" in r.stdout
