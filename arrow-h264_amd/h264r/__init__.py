"""h264r -- MI355X-native H.264 macroblock reconstruction, host API.

Python mirror of the reference's per-macroblock `vio::h264::Decoder` interface
(R/src/codec/h264/decoder/decoder.h:301-338) over the C ABI of
include/h264r.h.  Every call that produces samples runs the gfx950 kernels of
lib/libh264r.so; there is no CPU fallback: without the library or without a
gfx950 device the constructor raises.

    reference                               here
    Decoder::assign_quant_params(slice)     Decoder.assign_quant_params(quant)
    Decoder::init(slice)                    Decoder.init(width_mbs, height_mbs, pic, slices)
    Decoder::coeff_* / transform_*_dc       raw levels inside the per-MB level block
    Decoder::decode(mb)                     Decoder.decode(mb_addr, mb, levels, mv, ref_idx)
    Decoder::deblock_filter(slice)          Decoder.deblock_filter(keep_slot) -> (Y, Cb, Cr)
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _abi as A
from ._abi import MB_DTYPE, PIC_DTYPE, QUANT_DTYPE, SLICE_DTYPE  # noqa: F401

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("H264R_LIB") or os.path.join(PKG_DIR, "lib", "libh264r.so")


class H264RError(RuntimeError):
    def __init__(self, fn: str, status: int):
        msg = _lib.h264r_strerror(status).decode() if _lib is not None else str(status)
        super().__init__(f"{fn} -> {status} ({msg})")
        self.status = status


_lib: C.CDLL | None = None


def build() -> str:
    """Compile lib/libh264r.so for gfx950 (hipcc cross-compiles without a GPU)."""
    import subprocess
    subprocess.run(["make", "-s", "-j8", "-C", PKG_DIR], check=True)
    return LIB_PATH


def lib() -> C.CDLL:
    """The native library; raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} missing: run h264r.build() / `make -C arrow-h264_amd`")
    # One HIP runtime per process: torch ships its own libamdhip64 (SONAME
    # libamdhip64.so.7).  Loading torch first makes libh264r bind to that same
    # runtime, so torch tensors (device memory, streams, RCCL) and our kernels
    # share one device context.  Without torch the system ROCm runtime is used.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    P, I = C.c_void_p, C.c_int
    sig = {
        "h264r_abi_version": ([], I), "h264r_strerror": ([I], C.c_char_p),
        "h264r_device_count": ([], I), "h264r_quant_init_flat": ([P], I),
        "h264r_quant_init_lists": ([P, P], I),
        "h264r_create": ([C.POINTER(P), I, I, I, I, I], I), "h264r_destroy": ([P], I),
        "h264r_set_ref": ([P, I, P, P, P, I, I], I),
        "h264r_picture_begin": ([P, I, I, P, P, P], I),
        "h264r_mb_submit": ([P, I, P, P, I, P, P], I),
        "h264r_picture_end": ([P, P, P, P, I], I),
        "h264r_picture_end_async": ([P, I], I),
        "h264r_picture_wait": ([P, P, P, P], I),
        "h264r_decode_batch": ([P, C.POINTER(A.Batch), P], I),
        "h264r_decode_batch_rows": ([P, C.POINTER(A.Batch), I, I, P], I),
        "h264r_ref_planes": ([P, I, C.POINTER(P), C.POINTER(P), C.POINTER(P)], I),
        "h264r_last_timing": ([P, C.POINTER(C.c_float)], I),
        "h264r_set_timing": ([P, I], I), "h264r_set_debug": ([P, I], I),
        "h264r_check": ([P], I),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes, f.restype = args, res
    A.bind_synth(L)
    from .group import bind as bind_group
    bind_group(L)
    if L.h264r_abi_version() != A.ABI_VERSION:
        raise ImportError("libh264r ABI version mismatch")
    _lib = L
    return L


def _check(fn: str, st: int) -> None:
    if st != A.OK:
        raise H264RError(fn, st)


def device_count() -> int:
    return int(lib().h264r_device_count())


def quant_flat() -> np.ndarray:
    q = np.zeros(1, QUANT_DTYPE)
    _check("h264r_quant_init_flat", lib().h264r_quant_init_flat(A.ptr(q)))
    return q


def quant_lists(m4: np.ndarray, m8: np.ndarray) -> np.ndarray:
    """h264r_quant_init_lists from resolved scaling matrices: m4 [6][16] (Intra Y/Cb/Cr, Inter
    Y/Cb/Cr), m8 [6][64] (Intra Y, Inter Y, Intra Cb, Inter Cb, Intra Cr, Inter Cr), raster."""
    m4 = np.ascontiguousarray(m4, np.int32).reshape(6, 16)
    m8 = np.ascontiguousarray(m8, np.int32).reshape(6, 64)
    arr = (C.c_void_p * 12)(*([m4[i].ctypes.data for i in range(6)] + [m8[i].ctypes.data for i in range(6)]))
    q = np.zeros(1, QUANT_DTYPE)
    _check("h264r_quant_init_lists", lib().h264r_quant_init_lists(A.ptr(q), arr))
    return q


class Decoder:
    """One reconstruction context on one GPU (reference: one Decoder per slice_t)."""

    def __init__(self, device: int = 0, max_width_mbs: int = 240, max_height_mbs: int = 135, chroma_format: int = 1):
        L = lib()
        h = C.c_void_p()
        _check("h264r_create", L.h264r_create(C.byref(h), device, max_width_mbs, max_height_mbs, chroma_format, 8))
        self._fmt = chroma_format
        self._h = h
        self._L = L
        self._quant = quant_flat()
        self._dims = None

    # -- lifetime -------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.h264r_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    # -- reference-shaped API -------------------------------------------------------
    def assign_quant_params(self, quant: np.ndarray) -> None:
        """Decoder::assign_quant_params: InvLevelScale tables for the next pictures."""
        self._quant = np.ascontiguousarray(quant, QUANT_DTYPE).reshape(1)

    def set_ref(self, slot: int, y: np.ndarray, u: np.ndarray, v: np.ndarray) -> None:
        H, W = y.shape
        _check("h264r_set_ref", self._L.h264r_set_ref(
            self._h, slot, A.ptr(np.ascontiguousarray(y)), A.ptr(np.ascontiguousarray(u)),
            A.ptr(np.ascontiguousarray(v)), W // 16, H // 16))

    def init(self, width_mbs: int, height_mbs: int, pic: np.ndarray, slices: np.ndarray) -> None:
        """Decoder::init + picture start (slice_data.cc:595-634)."""
        self._pic = np.ascontiguousarray(pic, PIC_DTYPE).reshape(1)
        self._slices = np.ascontiguousarray(slices, SLICE_DTYPE)
        _check("h264r_picture_begin", self._L.h264r_picture_begin(
            self._h, width_mbs, height_mbs, A.ptr(self._pic), A.ptr(self._slices), A.ptr(self._quant)))
        self._dims = (width_mbs, height_mbs)

    def decode(self, mb_addr: int, mb: np.ndarray, levels: np.ndarray, mv: np.ndarray,
               ref_idx: np.ndarray) -> None:
        """Decoder::decode(mb): mb is one MB_DTYPE record, levels its level block,
        mv uint32[2,16] and ref_idx int8[2,16] its 4x4 motion entries (raster)."""
        rec = np.ascontiguousarray(mb, MB_DTYPE).reshape(1)
        lv = np.ascontiguousarray(levels, np.int16)
        mvv = np.ascontiguousarray(mv, np.uint32).reshape(2, 16)
        rr = np.ascontiguousarray(ref_idx, np.int8).reshape(2, 16)
        _check("h264r_mb_submit", self._L.h264r_mb_submit(
            self._h, mb_addr, A.ptr(rec), A.ptr(lv) if lv.size else None, int(lv.size), A.ptr(mvv), A.ptr(rr)))

    def deblock_filter(self, keep_slot: int = -1):
        """Decoder::deblock_filter: runs reconstruction + deblocking for the picture on
        the GPU and returns the (Y, Cb, Cr) planes."""
        W, H = self._dims
        cw, ch = A.chroma_mb(self._fmt)
        y = np.empty((16 * H, 16 * W), np.uint8)
        u = np.empty((ch * H, cw * W), np.uint8)
        v = np.empty((ch * H, cw * W), np.uint8)
        _check("h264r_picture_end", self._L.h264r_picture_end(self._h, A.ptr(y), A.ptr(u), A.ptr(v), keep_slot))
        return y, u, v

    def deblock_filter_async(self, keep_slot: int = -1) -> None:
        """h264r_picture_end_async: the picture is reconstructed while the caller stages
        the next one; its planes come from wait() (oldest first)."""
        _check("h264r_picture_end_async", self._L.h264r_picture_end_async(self._h, keep_slot))
        self._waiting = getattr(self, "_waiting", []) + [self._dims]

    def wait(self):
        """h264r_picture_wait: planes of the oldest picture handed to deblock_filter_async."""
        W, H = self._waiting.pop(0)
        cw, ch = A.chroma_mb(self._fmt)
        y = np.empty((16 * H, 16 * W), np.uint8)
        u = np.empty((ch * H, cw * W), np.uint8)
        v = np.empty((ch * H, cw * W), np.uint8)
        _check("h264r_picture_wait", self._L.h264r_picture_wait(self._h, A.ptr(y), A.ptr(u), A.ptr(v)))
        return y, u, v

    def set_debug(self, flags: int) -> None:
        _check("h264r_set_debug", self._L.h264r_set_debug(self._h, flags))

    # -- convenience ----------------------------------------------------------------
    def decode_picture(self, p, refs=None, keep_slot: int = -1, no_deblock: bool = False,
                       intra_walk: bool = False, debug: int = 0):
        """Submit every MB of a synth.Picture (raster order) and return its planes
        (debug: further h264r_set_debug flags for this picture)."""
        from .mbview import iter_mbs
        if refs is not None:
            for s, (y, u, v) in enumerate(refs):
                self.set_ref(s, y, u, v)
        W, H = p.cfg.width_mbs, p.cfg.height_mbs
        self.init(W, H, p.pic, p.slices)
        for addr, rec, lv, mv, rr in iter_mbs(p):
            self.decode(addr, rec, lv, mv, rr)
        self.set_debug((A.DBG_NO_DEBLOCK if no_deblock else 0) | (A.DBG_INTRA_WALK if intra_walk else 0) | debug)
        try:
            return self.deblock_filter(keep_slot)
        finally:
            self.set_debug(0)

    def ref_planes(self, slot: int):
        y, u, v = C.c_void_p(), C.c_void_p(), C.c_void_p()
        _check("h264r_ref_planes", self._L.h264r_ref_planes(self._h, slot, C.byref(y), C.byref(u), C.byref(v)))
        return y.value, u.value, v.value

    def decode_batch(self, batch: A.Batch, stream: int | None = None, rows: tuple[int, int] | None = None) -> None:
        """Reconstruct + deblock every picture of a device-resident batch; with `rows` =
        (row0, row1) only that slice-aligned band of MB rows (h264r_decode_batch_rows)."""
        if rows is None:
            _check("h264r_decode_batch", self._L.h264r_decode_batch(self._h, C.byref(batch), C.c_void_p(stream or 0)))
        else:
            _check("h264r_decode_batch_rows", self._L.h264r_decode_batch_rows(
                self._h, C.byref(batch), int(rows[0]), int(rows[1]), C.c_void_p(stream or 0)))

    def check(self) -> None:
        """Synchronise and raise if a device-side wavefront wait timed out."""
        _check("h264r_check", self._L.h264r_check(self._h))

    def set_timing(self, on: bool) -> None:
        _check("h264r_set_timing", self._L.h264r_set_timing(self._h, 1 if on else 0))

    def last_timing(self):
        out = (C.c_float * 4)()
        _check("h264r_last_timing", self._L.h264r_last_timing(self._h, out))
        return [float(x) for x in out]
