#!/usr/bin/env python3
"""Generate tests/golden/golden.json from the compiled REFERENCE decoder.

Run in the container that holds /root/reference (the GPU box never does):

    python tests/golden/make_golden.py

For every case below, the seeded synthetic picture (arrow-h264_amd/csrc/synth.c)
is decoded by the unmodified reference (oracle/_ref/ref_driver, built from
/root/reference by oracle/Makefile: Decoder::coeff_* pushes, Decoder::decode per
MB in raster order, Decoder::deblock_filter).  The fixture keeps:
  - the synth configuration and picture index (inputs are regenerated),
  - an MD5 of every generated input array (detects generator drift),
  - per-plane MD5 of the reconstruction before deblocking and of the final output
    (the reference's own compare protocol is per-frame MD5 of the YUV,
     R/script/test/model/__init__.py:119-183).
The script also checks the oracle restatement against the reference bytes and
refuses to write fixtures if they differ.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402

import _oracle as O  # noqa: E402
from h264r import synth  # noqa: E402

# name, SURVEY config index, W, H, overrides, picture indices
CASES = [
    ("intra_qcif", 2, 11, 9, dict(pcm_permille=20), [0, 1, 2]),
    ("intra_qcif_4x4only", 2, 11, 9, dict(transform8x8=0), [0]),
    ("intra_cif_3slices_idc2", 2, 22, 18, dict(num_slices=3, deblock_idc=2, pcm_permille=10), [0]),
    ("intra_cif_3slices_idc0", 2, 22, 18, dict(num_slices=3, deblock_idc=0), [0]),
    ("intra_qcif_offsets", 2, 11, 9, dict(filter_offset_a=12, filter_offset_b=-12), [0]),
    ("intra_qcif_lowqp", 2, 11, 9, dict(qp_min=0, qp_max=15), [0]),
    ("intra_qcif_highqp", 2, 11, 9, dict(qp_min=40, qp_max=51), [0]),
    ("p_qcif", 3, 11, 9, {}, [0, 1, 2]),
    ("p_qcif_wp", 3, 11, 9, dict(wp_mode=1), [0, 1]),
    ("p_qcif_cip", 3, 11, 9, dict(constrained_intra=1, intra_permille=400), [0, 1]),
    ("p_qcif_idc1", 3, 11, 9, dict(deblock_idc=1), [0]),
    ("p_qcif_3slices_idc2", 3, 11, 9, dict(num_slices=3, deblock_idc=2), [0]),
    ("p_qcif_3slices_idc0", 3, 11, 9, dict(num_slices=3, deblock_idc=0), [0]),
    ("p_qcif_bigmv", 3, 11, 9, dict(mv_range_x=300, mv_range_y=200), [0, 1]),
    ("p_qcif_4refs_t8", 3, 11, 9, dict(num_refs=4, transform8x8=1), [0]),
    ("p_qcif_offsets", 3, 11, 9, dict(filter_offset_a=-6, filter_offset_b=8), [0]),
    ("p_qcif_pcm_highqp", 3, 11, 9, dict(pcm_permille=100, intra_permille=300, qp_min=36, qp_max=51), [0]),
    ("b_qcif_implicit", 4, 11, 9, dict(num_slices=1, deblock_idc=0), [0, 1]),
    ("b_qcif_default", 4, 11, 9, dict(wp_mode=0), [0]),
    ("b_qcif_explicit", 4, 11, 9, dict(wp_mode=1), [0, 1]),
    ("b_qcif_4refs", 4, 11, 9, dict(num_refs=4), [0]),
    ("b_qcif_bigmv_cip", 4, 11, 9, dict(mv_range_x=250, mv_range_y=150, constrained_intra=1), [0]),
    ("b_cif_4slices", 4, 22, 18, {}, [0]),
    ("p_1080p_strip", 3, 120, 4, {}, [0]),
    ("intra_1080p", 2, 120, 68, {}, [0]),
    ("p_1080p", 3, 120, 68, {}, [0]),
    ("b_1080p_4slices", 4, 120, 68, {}, [0]),
    ("b_2160p_strip", 5, 240, 8, dict(num_slices=2), [0]),
    # lossless (qpprime_y_zero_transform_bypass_flag, TransformBypassModeFlag MBs; F12)
    ("intra_qcif_lossless", 2, 11, 9, dict(qp_min=0, qp_max=30, lossless_permille=400, pcm_permille=20), [0, 1]),
    ("intra_qcif_lossless_4x4", 2, 11, 9, dict(qp_min=0, qp_max=10, transform8x8=0, lossless_permille=300), [0]),
    ("p_qcif_lossless_t8", 3, 11, 9, dict(qp_min=0, qp_max=30, lossless_permille=400, transform8x8=1,
                                          intra_permille=300), [0, 1]),
    ("b_qcif_lossless", 4, 11, 9, dict(qp_min=0, qp_max=20, lossless_permille=500), [0]),
    # SP slices (inverse_transform_sp transform.cc:1267-1300; F13): switching and not, QsY 0..5
    ("p_qcif_sp", 3, 11, 9, dict(sp_slices=1), [0, 1, 2]),
    ("p_cif_sp_3slices", 3, 22, 18, dict(sp_slices=1, num_slices=3, deblock_idc=2, intra_permille=200), [0]),
    ("p_qcif_sp_qp0_51", 3, 11, 9, dict(sp_slices=1, qp_min=0, qp_max=51, num_refs=3), [0, 1]),
    # explicit scaling matrices (SPS lists, all present; Transform::init/set_quant transform.cc:173-302)
    ("intra_qcif_scaling", 2, 11, 9, dict(qm=14), [0]),
    ("p_qcif_scaling_t8", 3, 11, 9, dict(transform8x8=1, qm=15), [0]),
    ("b_qcif_scaling", 4, 11, 9, dict(qm=11), [0]),
    ("b_1080p_4slices_scaling", 4, 120, 68, dict(qm=12), [0]),
    ("b_2160p_strip_scaling", 5, 240, 8, dict(num_slices=2, qm=13), [0]),
    # field pictures (PAFF; include/h264r.h H264R_TOP_FIELD): H is the field's MB rows, the
    # references are fields of DPB frames of 2H rows (both parities, chroma offset
    # inter_prediction.cc:352-355), mvlimit 2 and bS 3 on horizontal MB edges (deblock.cc:86-189)
    ("ifield_cif_top", 2, 22, 9, dict(structure=1, pcm_permille=20), [0]),
    ("ifield_cif_bottom_4x4_cip", 2, 22, 9, dict(structure=2, transform8x8=0, constrained_intra=1), [0]),
    ("pfield_cif_top", 3, 22, 9, dict(structure=1, num_refs=4), [0, 1]),
    ("pfield_cif_bottom_pcm", 3, 22, 9, dict(structure=2, num_refs=3, pcm_permille=30, intra_permille=200), [0, 1]),
    ("pfield_qcif_wp_bottom", 3, 11, 4, dict(structure=2, wp_mode=1, num_refs=4), [0]),
    ("pfield_cif_cip_3slices_idc2", 3, 22, 9, dict(structure=1, constrained_intra=1, intra_permille=400,
                                                   num_slices=3, deblock_idc=2), [0]),
    ("pfield_cif_sp", 3, 22, 9, dict(structure=2, sp_slices=1, num_refs=2), [0]),
    ("bfield_cif_top_implicit", 4, 22, 9, dict(structure=1, num_refs=4, num_slices=2), [0, 1]),
    ("bfield_cif_bottom_explicit", 4, 22, 9, dict(structure=2, wp_mode=1, num_refs=6), [0]),
    ("bfield_cif_bottom_bigmv", 4, 22, 9, dict(structure=2, wp_mode=0, mv_range_x=200, mv_range_y=100,
                                               num_slices=1, deblock_idc=0), [0]),
    ("bfield_qcif_lossless", 4, 11, 4, dict(structure=1, qp_min=0, qp_max=20, lossless_permille=500), [0]),
    ("pfield_1080i_top", 3, 120, 34, dict(structure=1), [0]),
    ("bfield_1080i_bottom_scaling", 4, 120, 34, dict(structure=2, qm=16), [0]),
    # 4:4:4 (chroma_format_idc 3, High 4:4:4 Predictive): every colour plane coded and decoded
    # like luma (decode_one_component decoder.cc:65-79), luma-style deblocking of Cb / Cr
    # (deblock.cc:422) with their QpC and the luma bS
    ("i444_qcif_pcm", 2, 11, 9, dict(chroma_format=3, pcm_permille=20), [0]),
    ("i444_qcif_4x4_cip", 2, 11, 9, dict(chroma_format=3, transform8x8=0, constrained_intra=1), [0]),
    ("p444_qcif", 3, 11, 9, dict(chroma_format=3, num_refs=2), [0, 1]),
    ("p444_cif_wp_pcm", 3, 22, 9, dict(chroma_format=3, wp_mode=1, num_refs=3, pcm_permille=30, intra_permille=200), [0]),
    ("b444_qcif_t8", 4, 11, 9, dict(chroma_format=3, num_refs=3), [0, 1]),
    ("b444_cif_explicit_3slices_idc2", 4, 22, 9, dict(chroma_format=3, wp_mode=1, num_refs=4, num_slices=3,
                                                     deblock_idc=2), [0]),
    ("p444_qcif_lossless", 3, 11, 9, dict(chroma_format=3, qp_min=0, qp_max=20, lossless_permille=500), [0]),
    ("b444_qcif_scaling", 4, 11, 9, dict(chroma_format=3, qm=17), [0]),
    ("p444_1080p_strip_qp", 3, 120, 6, dict(chroma_format=3, qp_min=0, qp_max=51, num_slices=2), [0]),
    # 4:2:2 (chroma_format_idc 2, High 4:2:2): 8 x 16 chroma per MB, the 2x4 chroma DC
    # (transform.cc:890-908, qp_scaled as the reference has it), the plane constants yCF 4
    # (intra_prediction.cc:871-894), quarter-row chroma vectors (inter_prediction.cc:381-383), four
    # horizontal chroma edges (deblock.cc:273-274).  No 8x8 transforms: the reference leaves the bS
    # of a transform-8x8 MB's chroma rows 4 / 12 unset (h264r_oracle.c strength), the fixtures keep
    # to what it defines
    ("i422_qcif_pcm", 2, 11, 9, dict(chroma_format=2, transform8x8=0, pcm_permille=30), [0, 1]),
    ("i422_qcif_cip_highqp", 2, 11, 9, dict(chroma_format=2, transform8x8=0, constrained_intra=1, qp_min=30,
                                            qp_max=51), [0]),
    ("p422_qcif", 3, 11, 9, dict(chroma_format=2, num_refs=2), [0, 1]),
    ("p422_cif_wp_pcm", 3, 22, 9, dict(chroma_format=2, wp_mode=1, num_refs=3, pcm_permille=30, intra_permille=200), [0]),
    ("p422_qcif_cip_bigmv", 3, 11, 9, dict(chroma_format=2, constrained_intra=1, intra_permille=400, mv_range_x=200,
                                           mv_range_y=120), [0]),
    ("b422_qcif_implicit", 4, 11, 9, dict(chroma_format=2, transform8x8=0, num_refs=3), [0, 1]),
    ("b422_cif_explicit_3slices_idc2", 4, 22, 9, dict(chroma_format=2, transform8x8=0, wp_mode=1, num_refs=4,
                                                     num_slices=3, deblock_idc=2), [0]),
    ("p422_qcif_lossless", 3, 11, 9, dict(chroma_format=2, qp_min=0, qp_max=20, lossless_permille=500), [0]),
    ("b422_qcif_scaling", 4, 11, 9, dict(chroma_format=2, transform8x8=0, qm=18), [0]),
    ("p422_1080p_strip_qp", 3, 120, 6, dict(chroma_format=2, qp_min=0, qp_max=51, num_slices=2), [0]),
    # 4:0:0 (chroma_format_idc 0, High): the luma alone -- no chroma prediction, residual or deblocking
    # (decoder.cc:199, deblock.cc:498,522); a PCM MB carries 256 samples
    ("i400_qcif_pcm_t8", 2, 11, 9, dict(chroma_format=4, pcm_permille=30), [0]),
    ("p400_qcif_wp_cip", 3, 11, 9, dict(chroma_format=4, wp_mode=1, num_refs=2, constrained_intra=1,
                                         intra_permille=300), [0, 1]),
    ("b400_cif_3slices_idc2", 4, 22, 9, dict(chroma_format=4, num_refs=3, num_slices=3, deblock_idc=2), [0]),
    ("p400_qcif_lossless", 3, 11, 9, dict(chroma_format=4, qp_min=0, qp_max=20, lossless_permille=500), [0]),
    # MBAFF frames (MbaffFrameFlag, structure 3): frame and field MB pairs at random; field MBs predict
    # from fields (get_ref_pic dpb.cc:1046-1055) with field block rows and the chroma parity offset
    # (inter_prediction.cc:356-361,470-474), intra neighbours where get_neighbour finds them
    # (neighbour.cc:123-173), MbAffPostProc and the mixed-edge loop filter (deblock.cc:78-289,418-629)
    ("imbaff_qcif_pcm", 2, 11, 8, dict(structure=3, pcm_permille=30), [0, 1]),
    ("imbaff_cif_4x4_cip_2slices_idc2", 2, 22, 18, dict(structure=3, transform8x8=0, constrained_intra=1,
                                                        num_slices=2, deblock_idc=2), [0]),
    ("pmbaff_qcif", 3, 11, 8, dict(structure=3, num_refs=3), [0, 1]),
    ("pmbaff_cif_wp_cip_pcm", 3, 22, 18, dict(structure=3, wp_mode=1, num_refs=2, constrained_intra=1,
                                              intra_permille=300, pcm_permille=30), [0]),
    ("pmbaff_qcif_bigmv_offsets", 3, 11, 8, dict(structure=3, mv_range_x=200, mv_range_y=120,
                                                 filter_offset_a=6, filter_offset_b=-6), [0]),
    ("bmbaff_qcif_default_t8", 4, 11, 8, dict(structure=3, wp_mode=0, num_refs=3), [0, 1]),
    ("bmbaff_cif_explicit_3slices_idc2", 4, 22, 18, dict(structure=3, wp_mode=1, num_refs=4, num_slices=3,
                                                         deblock_idc=2), [0]),
    ("bmbaff_qcif_scaling_idc1", 4, 11, 8, dict(structure=3, wp_mode=0, deblock_idc=1, qm=19), [0]),
    ("pmbaff_1080p_strip", 3, 120, 8, dict(structure=3, qp_min=10, qp_max=51), [0]),
]


# separate colour planes (JV, separate_colour_plane_flag, High 4:4:4): each colour plane of the frame is
# a monochrome picture with its own MBs, decoded with that plane's scaling lists and from that plane of
# the 4:4:4 references; ref_driver drives the unmodified reference's JV decode + deblock +
# make_frame_picture_JV (deblock.cc:555-579, 641-655).  Scaling lists: the first entries of the three
# intra 4x4 lists agree (the reference scales an Intra_16x16 DC of every plane by the Y list,
# transform.cc:831-836)
JV_CASES = [
    ("jv_i_qcif_pcm", 2, 11, 9, dict(pcm_permille=20), [0, 1, 2]),
    ("jv_p_cif_2slices_idc2", 3, 22, 9, dict(num_refs=2, num_slices=2, deblock_idc=2), [0, 1, 2]),
    ("jv_p_qcif_wp_cip", 3, 11, 9, dict(wp_mode=1, num_refs=3, constrained_intra=1, intra_permille=300), [0, 1, 2]),
    ("jv_b_qcif_explicit_t8", 4, 11, 9, dict(wp_mode=1, num_refs=2), [0, 1, 2]),
    ("jv_b_qcif_scaling", 4, 11, 9, dict(num_refs=3, qm=22), [0, 1, 2]),
]


def jv_quant(qseed):
    """qmatrix(qseed) with the Cb / Cr intra 4x4 lists' first entry equal to the Y list's"""
    m4, m8 = O.qmatrix(qseed)
    m4 = np.array(m4).copy()
    m4[1][0] = m4[2][0] = m4[0][0]
    return m4, np.array(m8)


def md5(a: np.ndarray) -> str:
    return hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()


def main() -> int:
    if not O.reference_available():
        print("reference not available: fixtures cannot be regenerated here", file=sys.stderr)
        return 2
    L = O.lib()
    fixtures = []
    for name, cidx, W, H, over, indices in CASES:
        over = dict(over)
        qseed = over.pop("qm", None)
        cfg = synth.default_cfg(L, cidx, W, H, **over)
        qm = O.qmatrix(qseed) if qseed is not None else None
        quant = O.quant_lists(*qm) if qm is not None else None
        for idx in indices:
            t0 = time.time()
            p = synth.picture(L, cfg, idx)
            entry = {"name": name, "config": cidx, "cfg": cfg.as_dict(), "index": idx,
                     "input_md5": synth.input_digest(p)}
            if qm is not None:
                entry["qmatrix"] = {"m4": qm[0].tolist(), "m8": qm[1].tolist()}
            for stage, recon_only in (("recon", True), ("out", False)):
                ref = O.run_reference(cfg, idx, recon_only=recon_only, qm=qm)
                ora = O.decode(p, stage="recon" if recon_only else "full", quant=quant)
                for k, pl in enumerate("YUV"):
                    if not np.array_equal(ref[k], ora[k]):
                        bad = np.argwhere(ref[k] != ora[k])
                        print(f"MISMATCH {name}[{idx}] {stage} plane {pl}: {len(bad)} samples, "
                              f"first at (y,x)={tuple(bad[0])}", file=sys.stderr)
                        return 1
                entry[f"{stage}_md5"] = {pl: md5(ref[k]) for k, pl in enumerate("YUV")}
            fixtures.append(entry)
            print(f"{name}[{idx}] {W}x{H} ok ({time.time() - t0:.2f}s)")
    jv = []
    for name, cidx, W, H, over, planes in JV_CASES:
        over = dict(over)
        qseed = over.pop("qm", None)
        qm = jv_quant(qseed) if qseed is not None else None
        cfg = synth.default_cfg(L, cidx, W, H, chroma_format=4, seed=0x5E9C + cidx, **over)
        for k in planes:
            p = synth.picture(L, cfg, k)               # plane k: its own MBs (picture index k)
            ref = O.run_reference(cfg, k, qm=qm, jv_plane=k)
            ora = O.decode_jv_plane(p, k, qm)
            if not np.array_equal(ref, ora):
                bad = np.argwhere(ref != ora)
                print(f"MISMATCH {name} plane {k}: {len(bad)} samples, first at {tuple(bad[0])}", file=sys.stderr)
                return 1
            entry = {"name": name, "config": cidx, "cfg": cfg.as_dict(), "index": k, "colour_plane": k,
                     "input_md5": synth.input_digest(p), "out_md5": md5(ref)}
            if qm is not None:
                entry["qmatrix"] = {"m4": qm[0].tolist(), "m8": qm[1].tolist()}
            jv.append(entry)
            print(f"{name} plane {k} {W}x{H} ok")
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "reference": "luuvish/arrow-h264 decoder/*.cc compiled by oracle/Makefile",
                   "fixtures": fixtures, "jv_fixtures": jv}, f, indent=1)
    print(f"wrote {len(fixtures)} fixtures, {len(jv)} JV plane fixtures")
    return 0


if __name__ == "__main__":
    sys.exit(main())
