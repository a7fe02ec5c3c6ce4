"""Stream-level parity fixtures (TEST INFRASTRUCTURE).

SURVEY.md 8(c) items 2-3 and 8(f) rank 1.  A fixed set of H.264 streams written by the
repo's own bitstream writer (tests/h264_writer.py) is committed under
tests/golden/streams/, together with, per stream:

* the reference's per-frame MD5s of its decoded YUV: the unmodified reference decoder
  (oracle/_ref/ldecod, built from /root/reference) run in this container, digested with
  the reference harness's protocol (script/test/model/__init__.py:119-183,
  h264r.output.digest_by_frames);
* the MB records captured at the C-ABI boundary while the reference's own parser drives
  the drop-in Decoder shim (oracle/_ref/ldecod_shim, shim/decoder_h264r.cc): for every
  picture the h264r_mb records, level pool, motion, slice table, picture parameters,
  quantisation tables and DPB slot it is kept in (<name>.cap.npz).  The GPU tests
  replay them through libh264r.so, where the reference cannot run.

tests/golden/make_streams.py regenerates everything (this container only).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLDEN = os.path.join(HERE, "golden")
STREAM_DIR = os.path.join(GOLDEN, "streams")
STREAMS_JSON = os.path.join(GOLDEN, "streams.json")
sys.path.insert(0, os.path.join(ROOT, "arrow-h264_amd"))

from h264r import _abi as A  # noqa: E402
from h264r import output as OUT  # noqa: E402

# name -> tests/h264_writer.StreamCfg fields
STREAMS = {
    "bp_qcif_ippp": dict(width_mbs=11, height_mbs=9, frames=4, seed=101),
    "bp_qcif_slices_cip": dict(width_mbs=11, height_mbs=9, frames=5, seed=102, slices=3, deblock=(0, 1, 2),
                               offsets=6, num_refs=3, cip=1, chroma_qp_offset=-5),
    "bp_cif_wp_pcm": dict(width_mbs=22, height_mbs=18, frames=4, seed=103, weighted=1, num_refs=2, pcm=0.1,
                          skip=0.3),
    "bp_qcif_intra_qp0_51": dict(width_mbs=11, height_mbs=9, frames=3, seed=104, all_intra=True, qp=(0, 51),
                                 level_max=3),
    "hp_cif_8x8": dict(width_mbs=22, height_mbs=18, frames=4, seed=105, profile=100, transform8x8=1, slices=2,
                       deblock=(0, 2), offsets=3, chroma_qp_offset=4, second_chroma_qp_offset=-3),
    "hp_qcif_scaling_lists": dict(width_mbs=11, height_mbs=9, frames=4, seed=106, profile=100, transform8x8=1,
                                  scaling=3, qp=(10, 34)),
    "hp_qcif_scaling_pps_4x4": dict(width_mbs=11, height_mbs=9, frames=3, seed=107, profile=100, transform8x8=0,
                                    scaling=2),
    "bp_vga_crop_8slices": dict(width_mbs=40, height_mbs=30, frames=3, seed=108, crop=(1, 2, 0, 4), slices=8,
                                deblock=(0, 1, 2), offsets=6, intra_in_p=0.3, num_refs=2),
    "hi444_qcif_lossless": dict(width_mbs=11, height_mbs=9, frames=4, seed=110, profile=244, transform8x8=1,
                                lossless=0.5, qp=(0, 30), intra_in_p=0.4, deblock=(0, 2), offsets=4),
    "xp_qcif_sp": dict(width_mbs=11, height_mbs=9, frames=5, seed=111, profile=88, sp=0.8, num_refs=2,
                       intra_in_p=0.2, slices=2, deblock=(0, 1, 2), offsets=3),
    "hp_720p_4slices": dict(width_mbs=80, height_mbs=45, frames=2, seed=109, profile=100, transform8x8=1,
                            slices=4, deblock=(0, 2), scaling=1, num_refs=1),
    # B pictures (IBBP, output order != decoding order): temporal + spatial direct, B_8x8 with direct
    # sub-blocks, every B partition; default / implicit (POC distances) / explicit bi-prediction weights
    "mp_qcif_ibbp_direct": dict(width_mbs=11, height_mbs=9, frames=7, seed=201, profile=77, bframes=2, num_refs=3),
    "mp_qcif_ibbp_implicit": dict(width_mbs=11, height_mbs=9, frames=7, seed=202, profile=77, bframes=2, num_refs=3,
                                  direct=(1,), bipred=2),
    "hp_qcif_ibbp_explicit_8x8": dict(width_mbs=11, height_mbs=9, frames=7, seed=203, profile=100, transform8x8=1,
                                      bframes=2, num_refs=3, direct=(0,), bipred=1),
    "hp_cif_ibbbp_bref_slices": dict(width_mbs=22, height_mbs=18, frames=10, seed=205, profile=100, transform8x8=1,
                                     bframes=3, b_ref=0.5, direct=(1,), bipred=2, num_refs=4, slices=3,
                                     deblock=(0, 1, 2), offsets=4, cip=1, intra_in_p=0.15),
    # CABAC (entropy_coding_mode_flag 1, tests/h264_cabac.py): every cabac_init_idc, PCM inside CABAC
    # slices, 8x8 transform blocks as one 64-coefficient block (interpret_residual.cc:453-456)
    "mp_cif_cabac_ippp_slices": dict(width_mbs=22, height_mbs=18, frames=4, seed=401, profile=77, cabac=1, slices=3,
                                     deblock=(0, 1, 2), offsets=6, pcm=0.05, num_refs=2, weighted=1, cip=1),
    "hp_cif_cabac_ibbp_4slices": dict(width_mbs=22, height_mbs=18, frames=7, seed=402, profile=100, transform8x8=1,
                                      cabac=1, bframes=2, num_refs=3, bipred=2, slices=4, deblock=(2,), offsets=3),
    "hp_qcif_cabac_intra_qp0_51": dict(width_mbs=11, height_mbs=9, frames=2, seed=403, profile=100, transform8x8=1,
                                       cabac=1, all_intra=True, qp=(0, 51), pcm=0.05, level_max=3),
    "hp_cif_cabac_bref_explicit_scaling": dict(width_mbs=22, height_mbs=18, frames=8, seed=404, profile=100,
                                               transform8x8=1, cabac=1, bframes=3, b_ref=0.5, direct=(1,), bipred=1,
                                               num_refs=4, scaling=3, chroma_qp_offset=3, second_chroma_qp_offset=-2),
    # BASELINE config 4's shape as a real stream: 1080p High, IBBP, 8x8 transform, CABAC, 4 slices, idc 2
    "hp_1080p_cabac_ibbp_4slices": dict(width_mbs=120, height_mbs=68, frames=4, seed=405, profile=100, transform8x8=1,
                                        cabac=1, bframes=2, num_refs=3, bipred=2, slices=4, deblock=(2,), offsets=2,
                                        crop=(0, 0, 0, 4)),
    # 40 pictures with two long-term references (the IDR, and picture 2 by MMCO 4 + 6) used all
    # along: more reference pictures than device DPB slots over the stream's life
    "bp_qcif_longterm_40": dict(width_mbs=11, height_mbs=9, frames=40, seed=204, num_refs=4, long_term=2, skip=0.3,
                                intra_in_p=0.05),
    # field pictures (PAFF, frame_mbs_only_flag 0): every frame or a share of them as a top + bottom field
    # pair (some bottom first), P fields predicting from reference fields of both parities -- the first
    # field of their own frame too --, frame pictures predicting from frames decoded as field pairs
    "mp_cif_paff_cavlc": dict(width_mbs=22, height_mbs=18, frames=6, seed=501, profile=77, field=1.0, num_refs=3,
                              slices=2, deblock=(0, 2), offsets=3, intra_in_p=0.15, pcm=0.03),
    "hp_cif_paff_mixed_wp_8x8": dict(width_mbs=22, height_mbs=18, frames=8, seed=502, profile=100, transform8x8=1,
                                     field=0.5, bottom_first=0.4, num_refs=4, weighted=1, deblock=(0, 1, 2),
                                     offsets=4),
    "mp_cif_cabac_paff": dict(width_mbs=22, height_mbs=18, frames=6, seed=503, profile=77, cabac=1, field=0.7,
                              num_refs=3, slices=3, cip=1, pcm=0.04, deblock=(0, 2)),
    "hp_cif_cabac_paff_8x8_scaling": dict(width_mbs=22, height_mbs=18, frames=5, seed=504, profile=100,
                                          transform8x8=1, cabac=1, field=1.0, bottom_first=0.5, num_refs=2,
                                          scaling=1, qp=(12, 40)),
    # B field pictures (IBBP, pic_order_cnt_type 0): list 0 / list 1 of reference fields by POC, spatial
    # direct from co-located fields of frames coded as frames or as fields, non-reference and
    # reference B field pairs, default / implicit / explicit bi-prediction
    "mp_cif_paff_ibbp_spatial": dict(width_mbs=22, height_mbs=18, frames=7, seed=601, profile=77, field=1.0,
                                     bframes=2, num_refs=3, direct=(1,), slices=2, deblock=(0, 2), offsets=2),
    "hp_cif_cabac_paff_ibbp_implicit_bref": dict(width_mbs=22, height_mbs=18, frames=8, seed=602, profile=100,
                                                 transform8x8=1, cabac=1, field=0.6, bottom_first=0.4, bframes=2,
                                                 num_refs=3, direct=(1,), bipred=2, b_ref=0.5),
    "hp_cif_paff_ibbp_explicit": dict(width_mbs=22, height_mbs=18, frames=7, seed=603, profile=100, transform8x8=1,
                                      field=0.7, bframes=1, num_refs=2, direct=(1,), bipred=1),
    "hp_1080i_cabac_paff": dict(width_mbs=120, height_mbs=68, frames=2, seed=505, profile=100, transform8x8=1,
                                cabac=1, field=1.0, num_refs=2, slices=4, deblock=(0, 2), crop=(0, 0, 0, 2)),
    # MBAFF frames (mb_adaptive_frame_field_flag, CAVLC, I and P): frame and field MB pairs at random
    # (mb_field_decoding_flag in a pair's top MB, in its bottom MB after a skipped top MB, inferred from
    # the left / upper pair for a skipped pair), CAVLC nC / intra-mode prediction / motion vector and
    # P_Skip prediction over the pairs' geometric neighbours (neighbour.cc:123-173, interpret_mv.cc:
    # 60-104, 158-190), field MBs predicting from reference fields with refIdx over 2 x
    # num_ref_idx_active (a te() of one bit with one reference); first_mb_in_slice in pairs
    "hp_cif_mbaff_intra_pcm": dict(width_mbs=22, height_mbs=18, frames=3, seed=901, profile=100, transform8x8=1,
                                   mbaff=0.5, all_intra=True, pcm=0.05, slices=2, deblock=(0, 2), offsets=3),
    "mp_cif_mbaff_ippp_slices": dict(width_mbs=22, height_mbs=18, frames=6, seed=902, profile=77, mbaff=0.5,
                                     skip=0.3, num_refs=3, slices=3, deblock=(0, 1, 2), offsets=4, intra_in_p=0.2,
                                     pcm=0.03),
    "hp_cif_mbaff_wp_8x8_scaling": dict(width_mbs=22, height_mbs=18, frames=6, seed=903, profile=100,
                                        transform8x8=1, mbaff=0.6, skip=0.2, num_refs=4, weighted=1, scaling=3,
                                        chroma_qp_offset=2, qp=(14, 40)),
    "mp_qcif_mbaff_oneref_skips": dict(width_mbs=11, height_mbs=10, frames=8, seed=905, profile=77, mbaff=0.5,
                                       skip=0.5, num_refs=1, intra_in_p=0.1),
    "hp_vga_mbaff_ippp": dict(width_mbs=40, height_mbs=34, frames=5, seed=904, profile=100, transform8x8=1,
                              mbaff=0.5, skip=0.25, num_refs=2, slices=2, deblock=(0, 2), intra_in_p=0.15),
    # MBAFF with CABAC: mb_field_decoding_flag as a bin (ctxIdxInc from the left / upper pairs), the
    # skip flags' contexts with the pair's inferred flag, a skipped top MB reading its bottom MB's skip
    # flag (and the pair's flag) ahead (interpret_mb.cc:186-262), end_of_slice_flag after bottom MBs,
    # refIdx / mvd contexts across field and frame pairs (neighbour.cc:517-633), field MBs' significance
    # contexts and 8x8 position map
    "hp_cif_cabac_mbaff_ippp": dict(width_mbs=22, height_mbs=18, frames=6, seed=911, profile=100, transform8x8=1,
                                    cabac=1, mbaff=0.5, skip=0.3, num_refs=3, slices=2, deblock=(0, 2),
                                    intra_in_p=0.15, pcm=0.02, qp=(14, 40)),
    "mp_qcif_cabac_mbaff_skips": dict(width_mbs=11, height_mbs=10, frames=8, seed=912, profile=77, cabac=1,
                                      mbaff=0.5, skip=0.5, num_refs=1, intra_in_p=0.1, weighted=1),
    # 4:2:2 (chroma_format_idc 2; High 4:2:2 / High 4:4:4 Predictive, CAVLC): 8 x 16 chroma per MB, the
    # 2x4 chroma DC (coeff_token nC -2, total_zeros of 8), 8 chroma AC blocks per plane.  No 8x8
    # transforms: the reference leaves the bS of a transform-8x8 MB's chroma rows 4 / 12 unset
    # (DESIGN.md section 4e), so its output there is not defined
    "hi422_qcif_intra_qp0_51": dict(width_mbs=11, height_mbs=9, frames=3, seed=701, profile=122, chroma_format=2,
                                    all_intra=True, qp=(0, 51), pcm=0.05, cip=1, level_max=3),
    "hi422_cif_ibbp_slices": dict(width_mbs=22, height_mbs=18, frames=7, seed=702, profile=122, chroma_format=2,
                                  bframes=2, num_refs=3, bipred=2, weighted=1, slices=3, deblock=(0, 1, 2),
                                  offsets=3, intra_in_p=0.2, pcm=0.03, chroma_qp_offset=-3,
                                  second_chroma_qp_offset=4, crop=(1, 2, 3, 2)),
    "hi422_qcif_lossless": dict(width_mbs=11, height_mbs=9, frames=4, seed=703, profile=244, chroma_format=2,
                                lossless=0.5, qp=(0, 30), intra_in_p=0.4, deblock=(0, 2), offsets=4, scaling=2),
    # ... and CABAC: the 2x4 DC with CHROMA_DC_2x4's significance maps (interpret_residual.cc:336), the
    # coded_block_flag of 8 AC blocks per plane (neighbour.cc:690-740 with MbHeightC 16)
    "hi422_cif_cabac_ibbp": dict(width_mbs=22, height_mbs=18, frames=7, seed=704, profile=122, chroma_format=2,
                                 cabac=1, bframes=2, num_refs=3, bipred=1, slices=2, deblock=(0, 2), offsets=2,
                                 intra_in_p=0.2, pcm=0.04, cip=1, chroma_qp_offset=3),
    "hi422_qcif_cabac_intra_qp0_51": dict(width_mbs=11, height_mbs=9, frames=2, seed=705, profile=122,
                                          chroma_format=2, cabac=1, all_intra=True, qp=(0, 51), pcm=0.05,
                                          level_max=3),
    # 4:4:4 (chroma_format_idc 3, High 4:4:4 Predictive, CAVLC): Cb and Cr coded as luma (their own
    # CAVLC nC), no intra chroma mode, the 4:4:4 CBP table; lossless MBs and 8x8 transforms
    "hi444_cif_ippp_8x8": dict(width_mbs=22, height_mbs=18, frames=4, seed=801, profile=244, chroma_format=3,
                               transform8x8=1, num_refs=2, weighted=1, slices=2, deblock=(0, 1, 2), offsets=3,
                               pcm=0.03, intra_in_p=0.2, chroma_qp_offset=2, second_chroma_qp_offset=-4,
                               crop=(2, 1, 0, 3)),
    "hi444_qcif_ibbp_lossless_scaling": dict(width_mbs=11, height_mbs=9, frames=7, seed=802, profile=244,
                                             chroma_format=3, transform8x8=1, bframes=2, num_refs=3, bipred=2,
                                             lossless=0.4, qp=(0, 36), intra_in_p=0.3, scaling=3, cip=1),
    # 4:0:0 (chroma_format_idc 0, High): luma only -- no chroma mode, CBP chroma, residual, PCM samples
    # or chroma weights; the reference writes 128-valued 4:2:0 chroma beside it (WriteUV, output.cc:205)
    "hp400_cif_ippp_8x8_wp": dict(width_mbs=22, height_mbs=18, frames=4, seed=901, profile=100, chroma_format=0,
                                  transform8x8=1, num_refs=2, weighted=1, slices=2, deblock=(0, 1, 2), offsets=3,
                                  pcm=0.03, intra_in_p=0.2, crop=(3, 1, 2, 5)),
    "hp400_qcif_cabac_ibbp": dict(width_mbs=11, height_mbs=9, frames=7, seed=902, profile=100, chroma_format=0,
                                  transform8x8=1, cabac=1, bframes=2, num_refs=3, bipred=1, pcm=0.04,
                                  intra_in_p=0.3, cip=1, scaling=3),
}

CAP_MAGIC = 0x43523448
QUANT_BYTES = A.QUANT_DTYPE.itemsize


def stream_path(name: str) -> str:
    return os.path.join(STREAM_DIR, name + ".264")


def capture_path(name: str) -> str:
    return os.path.join(STREAM_DIR, name + ".cap.npz")


# streams the repo's own parser (arrow-h264_amd/parser) refuses: reference-parser captures only
PARSER_REFUSED = {"hp_cif_cabac_mbaff_ippp": "MBAFF coding with CABAC", "mp_qcif_cabac_mbaff_skips": "MBAFF coding with CABAC"}


def crop_of(cfg: dict) -> OUT.Crop:
    """The SPS crop of a stream; its vertical unit is two chroma rows when the stream may
    hold field pictures (frame_mbs_only_flag 0, CropUnitY = SubHeightC * 2)."""
    l, r, t, b = cfg.get("crop", (0, 0, 0, 0))
    return OUT.Crop(left=l, right=r, top=t, bottom=b, frame_mbs_only=0 if cfg.get("field") or cfg.get("mbaff") else 1)


def structure(p: dict) -> int:
    return int(p["pic"]["structure"][0])


def output_frames(pics: list[dict], outs: list) -> list:
    """The decoded frames in output order.  A field pair (two consecutive field pictures of
    opposite parity, as the writer sends them) becomes one frame of interleaved rows
    (dpb_combine_field_yuv, picture.cc:578-622) with the smaller of its POCs; frames are
    ordered by POC inside each IDR period (a new period at every POC 0 after the first frame)
    -- the order the reference's DPB writes them (dpb.cc output process)."""
    frames, i = [], 0
    while i < len(pics):
        st = structure(pics[i])
        if st in (A.FRAME, A.MBAFF_FRAME):
            frames.append((int(pics[i]["pic"]["poc"][0]), i, outs[i]))
            i += 1
            continue
        j = i + 1
        assert j < len(pics) and structure(pics[j]) == 3 - st, "an unpaired field"
        top, bot = (outs[i], outs[j]) if st == A.TOP_FIELD else (outs[j], outs[i])
        planes = []
        for t, b in zip(top, bot):
            f = np.empty((2 * t.shape[0], t.shape[1]), np.uint8)
            f[0::2], f[1::2] = t, b
            planes.append(f)
        frames.append((min(int(pics[i]["pic"]["poc"][0]), int(pics[j]["pic"]["poc"][0])), i, tuple(planes)))
        i += 2
    keys, period = [], 0
    for k, (poc, i, _) in enumerate(frames):
        if k and poc == 0:
            period += 1
        keys.append((period, poc, k))
    return [frames[k][2] for _, _, k in sorted(keys)]


def output_order(pics: list[dict]) -> list[int]:
    """Decoding-order indices of captured pictures in output order: POC order inside each
    IDR period (a new period at every POC 0 after the first picture) -- the order the
    reference's DPB writes them (dpb.cc output process)."""
    keys, period = [], 0
    for i, p in enumerate(pics):
        poc = int(p["pic"]["poc"][0])
        if i and poc == 0:
            period += 1
        keys.append((period, poc, i))
    return [k[2] for k in sorted(keys)]


def frame_md5s(planes, cfg: dict) -> list[str]:
    """Per-frame MD5 of cropped output frames (write_out_picture + digest_by_frames)."""
    geom = OUT.geometry(cfg["width_mbs"], cfg["height_mbs"], crop_of(cfg), cfg.get("chroma_format", 1))
    return [hashlib.md5(OUT.frame_bytes(y, u, v, geom)).hexdigest() for (y, u, v) in planes]


def read_capture_file(path: str) -> list[dict]:
    """Parse the raw capture written by oracle/h264r_cpu_abi.c (H264R_CAPTURE)."""
    raw = open(path, "rb").read()
    off, pics = 0, []
    while off < len(raw):
        hdr = np.frombuffer(raw, np.int32, 8, off)
        off += 32
        magic, W, H, ns, nl, keep, cf, ver = (int(v) for v in hdr[:8])
        assert magic == CAP_MAGIC, "capture: bad record"
        n = W * H
        cf = cf if ver == 1 else 1                 # header[7] 1: header[6] is chroma_format_idc
        cw, ch = A.chroma_mb(cf)

        def take(dtype, count):
            nonlocal off
            a = np.frombuffer(raw, dtype, count, off).copy()
            off += a.nbytes
            return a
        p = dict(W=W, H=H, keep=keep, chroma_format=cf)
        p["mbs"] = take(A.MB_DTYPE, n)
        p["levels"] = take(np.int16, nl)
        p["mv"] = take(np.uint32, 2 * 16 * n).reshape(2, 4 * H, 4 * W)
        p["ref_idx"] = take(np.int8, 2 * 16 * n).reshape(2, 4 * H, 4 * W)
        p["slices"] = take(A.SLICE_DTYPE, ns)
        p["pic"] = take(A.PIC_DTYPE, 1)
        p["quant"] = take(A.QUANT_DTYPE, 1)
        y = take(np.uint8, 256 * n).reshape(16 * H, 16 * W)
        u = take(np.uint8, cw * ch * n).reshape(ch * H, cw * W)
        v = take(np.uint8, cw * ch * n).reshape(ch * H, cw * W)
        p["plane_md5"] = [hashlib.md5(a.tobytes()).hexdigest() for a in (y, u, v)]
        pics.append(p)
    return pics


def save_capture(path: str, pics: list[dict]) -> None:
    arrs = {}
    for i, p in enumerate(pics):
        for k in ("mbs", "levels", "mv", "ref_idx", "slices", "pic", "quant"):
            a = p[k]
            arrs[f"{i}_{k}"] = a.view(np.uint8) if a.dtype.names else a
        arrs[f"{i}_meta"] = np.array([p["W"], p["H"], p["keep"], p.get("chroma_format", 1)], np.int32)
        arrs[f"{i}_plane_md5"] = np.array(p["plane_md5"])
    np.savez_compressed(path, n=np.array([len(pics)]), **arrs)


def load_capture(path: str) -> list[dict]:
    z = np.load(path, allow_pickle=False)
    dt = {"mbs": A.MB_DTYPE, "slices": A.SLICE_DTYPE, "pic": A.PIC_DTYPE, "quant": A.QUANT_DTYPE}
    pics = []
    for i in range(int(z["n"][0])):
        meta = [int(v) for v in z[f"{i}_meta"]]
        W, H, keep = meta[:3]
        p = dict(W=W, H=H, keep=keep, chroma_format=meta[3] if len(meta) > 3 else 1)
        for k in ("mbs", "levels", "mv", "ref_idx", "slices", "pic", "quant"):
            a = z[f"{i}_{k}"]
            p[k] = a.view(dt[k]) if k in dt else a
        p["plane_md5"] = [str(s) for s in z[f"{i}_plane_md5"]]
        pics.append(p)
    return pics


def golden() -> dict:
    return json.load(open(STREAMS_JSON))


def iter_mbs(p: dict):
    """(addr, record, levels, mv[2,16], ref_idx[2,16]) of every MB of a captured picture,
    in the form Decoder.decode / h264r_mb_submit take."""
    W, H = p["W"], p["H"]
    mv = p["mv"].reshape(2, H, 4, W, 4).transpose(0, 1, 3, 2, 4).reshape(2, H * W, 16)
    ri = p["ref_idx"].reshape(2, H, 4, W, 4).transpose(0, 1, 3, 2, 4).reshape(2, H * W, 16)
    mbs = p["mbs"]
    offs = mbs["coef_off"].astype(np.int64)
    order = np.argsort(offs, kind="stable")
    ends = np.empty_like(offs)
    ends[order] = np.append(offs[order][1:], len(p["levels"]))
    for a in range(W * H):
        rec = mbs[a:a + 1].copy()
        rec["coef_off"] = 0
        yield a, rec, p["levels"][offs[a]:ends[a]], mv[:, a], ri[:, a]
