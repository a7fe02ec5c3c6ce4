"""ctypes / numpy mirror of include/h264r.h and include/h264r_synth.h.

Pure data-layout definitions shared by the host API (h264r/__init__.py), the
benchmark and the tests.  No behaviour lives here.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

# ---- constants (include/h264r.h) -------------------------------------------------
OK, EINVAL, ENOMEM, EDEVICE, ESTATE, EUNSUPPORTED, ENODEVICE = 0, -1, -2, -3, -4, -5, -6
DBG_NO_DEBLOCK, DBG_INTRA_WALK, DBG_DEBLOCK_MB, DBG_DEBLOCK_ROWS, DBG_DEBLOCK_GLOBAL = 1, 2, 4, 8, 16   # h264r_set_debug flags (include/h264r.h)
DBG_WAIT_TEST = 32
DBG_OVERLAP = 64
DBG_DEBLOCK_SPLIT = 128
MAX_REFS, MAX_SLOTS, MAX_SLICES = 16, 32, 256
ABI_VERSION = 4
FRAME, TOP_FIELD, BOTTOM_FIELD, MBAFF_FRAME = 0, 1, 2, 3   # h264r_pic.structure
REF_BOTTOM = 0x40                              # ref_slot entry of a field picture: the slot's bottom field

P_SKIP, P_16x16, P_16x8, P_8x16, P_8x8, P_8x4, P_4x8, P_4x4 = range(8)
I_4x4, I_8x8, I_16x16, SI, I_PCM = 8, 9, 10, 11, 12
SLICE_P, SLICE_B, SLICE_I, SLICE_SP, SLICE_SI = range(5)
MBF_INTRA, MBF_T8x8, MBF_BYPASS, MBF_FIELD = 1, 2, 4, 8

SYNTH_INTRA, SYNTH_P, SYNTH_B = 0, 1, 2
SYNTH_MAX_LEVELS_PER_MB = 416
SYNTH_MAX_LEVELS_PER_MB_422 = 544
SYNTH_MAX_LEVELS_PER_MB_444 = 816


SYNTH_CHROMA_400 = 4            # h264r_synth_cfg.chroma_format of 4:0:0 (0, the default, is 4:2:0)


def idc_of(synth_chroma_format: int) -> int:
    """chroma_format_idc of a synth configuration's chroma_format (include/h264r_synth.h)."""
    return {2: 2, 3: 3, SYNTH_CHROMA_400: 0}.get(int(synth_chroma_format), 1)


def chroma_mb(chroma_format: int) -> tuple[int, int]:
    """(width, height) of one MB's chroma in samples by chroma_format_idc: 4:2:0 8 x 8, 4:2:2 8 x 16,
    4:4:4 16 x 16, 4:0:0 none."""
    return {0: (0, 0), 2: (8, 16), 3: (16, 16)}.get(int(chroma_format), (8, 8))


def max_levels_per_mb(chroma_format: int) -> int:
    return {2: SYNTH_MAX_LEVELS_PER_MB_422, 3: SYNTH_MAX_LEVELS_PER_MB_444}.get(int(chroma_format),
                                                                              SYNTH_MAX_LEVELS_PER_MB)

# ---- numpy dtypes of the canonical device formats ----------------------------------
MB_DTYPE = np.dtype([
    ("mb_type", "u1"), ("flags", "u1"), ("cbp", "u1"), ("qp_y", "i1"),
    ("qp_c", "i1", (2,)), ("i16_mode", "u1"), ("chroma_mode", "u1"),
    ("cbp_blks", "<u2"), ("slice", "<u2"), ("qp_scaled", "u1", (3,)), ("pad0", "u1"),
    ("coef_off", "<u4"), ("ipred", "u1", (8,)), ("pad1", "u1", (4,)),
])
assert MB_DTYPE.itemsize == 32

SLICE_DTYPE = np.dtype([
    ("slice_type", "u1"), ("deblock_idc", "u1"), ("filter_offset_a", "i1"),
    ("filter_offset_b", "i1"), ("wp_mode", "u1"), ("luma_log2_wd", "u1"),
    ("chroma_log2_wd", "u1"), ("num_ref", "u1", (2,)), ("qs_y", "u1"), ("sp_switch", "u1"),
    ("qs_c", "i1", (2,)), ("pad", "u1", (3,)),
    ("ref_slot", "i1", (2, MAX_REFS)), ("wp_weight", "i1", (2, MAX_REFS, 3)),
    ("wp_offset", "i1", (2, MAX_REFS, 3)), ("implicit_w1", "<i2", (MAX_REFS, MAX_REFS)),
])
assert SLICE_DTYPE.itemsize == 752

QUANT_DTYPE = np.dtype([("scale4x4", "<i2", (2, 3, 6, 16)), ("scale8x8", "<i2", (2, 3, 6, 64))])
assert QUANT_DTYPE.itemsize == 5760

PIC_DTYPE = np.dtype([("constrained_intra_pred", "<i4"), ("num_slices", "<i4"),
                      ("poc", "<i4"), ("structure", "<i4")])


class SynthCfg(C.Structure):
    _fields_ = [
        ("width_mbs", C.c_int32), ("height_mbs", C.c_int32), ("kind", C.c_int32),
        ("num_slices", C.c_int32), ("deblock_idc", C.c_int32),
        ("filter_offset_a", C.c_int32), ("filter_offset_b", C.c_int32),
        ("transform8x8", C.c_int32), ("wp_mode", C.c_int32),
        ("constrained_intra", C.c_int32), ("num_refs", C.c_int32),
        ("qp_min", C.c_int32), ("qp_max", C.c_int32), ("pcm_permille", C.c_int32),
        ("intra_permille", C.c_int32), ("mv_range_x", C.c_int32),
        ("mv_range_y", C.c_int32), ("lossless_permille", C.c_int32), ("sp_slices", C.c_int32),
        ("structure", C.c_int32), ("chroma_format", C.c_int32), ("seed", C.c_uint64),
    ]

    def as_dict(self) -> dict:
        return {name: int(getattr(self, name)) for name, _ in self._fields_}

    @classmethod
    def from_dict(cls, d: dict) -> "SynthCfg":
        c = cls()
        for k, v in d.items():
            setattr(c, k, int(v))
        return c


class Batch(C.Structure):
    """h264r_batch: device pointers of a resident batch."""
    _fields_ = [
        ("num_pics", C.c_int32), ("width_mbs", C.c_int32), ("height_mbs", C.c_int32),
        ("slice_stride", C.c_int32), ("mbs", C.c_void_p), ("levels", C.c_void_p),
        ("mv", C.c_void_p), ("ref_idx", C.c_void_p), ("slices", C.c_void_p),
        ("pics", C.c_void_p), ("quant", C.c_void_p), ("ref_planes", C.c_void_p),
        ("out_y", C.c_void_p), ("out_u", C.c_void_p), ("out_v", C.c_void_p),
        ("ref_planes_stride", C.c_int64), ("mbaff", C.c_int32), ("colour_plane", C.c_int32),
    ]


def ptr(a: np.ndarray) -> C.c_void_p:
    """Host pointer of a C-contiguous numpy array."""
    assert a.flags["C_CONTIGUOUS"]
    return C.c_void_p(a.ctypes.data)


def bind_synth(lib: C.CDLL) -> None:
    """Declare the h264r_synth_* prototypes on a library that exports them."""
    P = C.c_void_p
    lib.h264r_synth_default.argtypes = [C.POINTER(SynthCfg), C.c_int, C.c_int, C.c_int]
    lib.h264r_synth_picture.argtypes = [C.POINTER(SynthCfg), C.c_int, P, P,
                                        C.POINTER(C.c_int64), P, P, P, P]
    lib.h264r_synth_refpic.argtypes = [C.c_uint64, C.c_int, C.c_int, C.c_int, P, P, P]
    lib.h264r_synth_refpic_fmt.argtypes = [C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P]
    lib.h264r_synth_slot_poc.argtypes = [C.c_int]
    lib.h264r_synth_cur_poc.argtypes = [C.POINTER(SynthCfg)]
    lib.h264r_synth_ref_frames.argtypes = [C.POINTER(SynthCfg)]
    lib.h264r_synth_algo_bytes.argtypes = [P, P, C.c_int, C.c_int,
                                           C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    for f in ("h264r_synth_default", "h264r_synth_picture", "h264r_synth_refpic", "h264r_synth_refpic_fmt",
              "h264r_synth_slot_poc", "h264r_synth_cur_poc", "h264r_synth_ref_frames", "h264r_synth_algo_bytes"):
        getattr(lib, f).restype = C.c_int
