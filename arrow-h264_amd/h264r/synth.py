"""Numpy front-end of the seeded synthetic workload (include/h264r_synth.h).

The generator itself is C (arrow-h264_amd/csrc/synth.c) so that the GPU
inputs, the CPU baseline and the reference-fixture driver see byte-identical
data; this module only allocates arrays and calls it through any library that
exports the h264r_synth_* symbols.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _abi as A


@dataclass
class Picture:
    cfg: A.SynthCfg
    index: int
    mbs: np.ndarray       # MB_DTYPE [H*W]
    levels: np.ndarray    # int16 pool (trimmed)
    mv: np.ndarray        # uint32 [2, 4H, 4W]
    ref_idx: np.ndarray   # int8 [2, 4H, 4W]
    slices: np.ndarray    # SLICE_DTYPE [num_slices]
    pic: np.ndarray       # PIC_DTYPE [1]


def default_cfg(lib: C.CDLL, config_idx: int, width_mbs: int, height_mbs: int, **over) -> A.SynthCfg:
    cfg = A.SynthCfg()
    st = lib.h264r_synth_default(C.byref(cfg), config_idx, width_mbs, height_mbs)
    if st != A.OK:
        raise ValueError(f"h264r_synth_default({config_idx}) -> {st}")
    for k, v in over.items():
        setattr(cfg, k, int(v))
    return cfg


def picture(lib: C.CDLL, cfg: A.SynthCfg, index: int) -> Picture:
    W, H = cfg.width_mbs, cfg.height_mbs
    n = W * H
    mbs = np.zeros(n, A.MB_DTYPE)
    idc = A.idc_of(cfg.chroma_format)
    levels = np.zeros(n * A.max_levels_per_mb(idc), np.int16)
    mv = np.zeros((2, 4 * H, 4 * W), np.uint32)
    ref_idx = np.zeros((2, 4 * H, 4 * W), np.int8)
    slices = np.zeros(cfg.num_slices, A.SLICE_DTYPE)
    pic = np.zeros(1, A.PIC_DTYPE)
    nlev = C.c_int64(0)
    st = lib.h264r_synth_picture(C.byref(cfg), index, A.ptr(mbs), A.ptr(levels), C.byref(nlev),
                                 A.ptr(mv), A.ptr(ref_idx), A.ptr(slices), A.ptr(pic))
    if st != A.OK:
        raise ValueError(f"h264r_synth_picture -> {st}")
    # 4:4:4: a PCM MB's Cr view reads 128 entries past its 384, 4:0:0 its chroma view 64 past its 128
    # (include/h264r.h): kept readable
    keep = max(int(nlev.value), 8) + (128 if idc == 3 else 64 if idc == 0 else 0)
    return Picture(cfg, index, mbs, levels[:keep].copy(), mv, ref_idx, slices, pic)


def refpics(lib: C.CDLL, cfg: A.SynthCfg, nslots: int | None = None):
    """[(y, u, v)] for DPB slots 0..n-1: the frames the pictures reference (a field cfg's
    references are fields of frames of twice its height, include/h264r_synth.h)."""
    W, H = cfg.width_mbs, cfg.height_mbs * (2 if cfg.structure in (A.TOP_FIELD, A.BOTTOM_FIELD) else 1)
    cw, ch = A.chroma_mb(A.idc_of(cfg.chroma_format))
    out = []
    for s in range(lib.h264r_synth_ref_frames(C.byref(cfg)) if nslots is None else nslots):
        y = np.zeros((16 * H, 16 * W), np.uint8)
        u = np.zeros((ch * H, cw * W), np.uint8)
        v = np.zeros((ch * H, cw * W), np.uint8)
        st = lib.h264r_synth_refpic_fmt(C.c_uint64(cfg.seed), s, W, H, int(cfg.chroma_format), A.ptr(y), A.ptr(u),
                                        A.ptr(v))
        if st != A.OK:
            raise ValueError(f"h264r_synth_refpic -> {st}")
        out.append((y, u, v))
    return out


def algo_bytes(lib: C.CDLL, p: Picture) -> tuple[int, int]:
    r, w = C.c_int64(0), C.c_int64(0)
    st = lib.h264r_synth_algo_bytes(A.ptr(p.mbs), A.ptr(p.ref_idx), p.cfg.width_mbs,
                                    p.cfg.height_mbs, C.byref(r), C.byref(w))
    if st != A.OK:
        raise ValueError(f"h264r_synth_algo_bytes -> {st}")
    return int(r.value), int(w.value)


def input_digest(p: Picture) -> str:
    """MD5 over every generated input array (detects generator drift vs fixtures)."""
    import hashlib
    h = hashlib.md5()
    for a in (p.mbs, p.levels, p.mv, p.ref_idx, p.slices, p.pic):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()
