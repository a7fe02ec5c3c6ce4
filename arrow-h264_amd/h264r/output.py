"""Output and compare step: the cropping YUV writer and the per-frame MD5 compare.

SURVEY §8(f) rank 3.  The reference writes every output picture as cropped
planar Y, Cb, Cr (`write_out_picture`, src/codec/h264/framebuf/output.cc:109-227)
and its test harness splits the decoded file into N equal frames, MD5s each and
compares count and digests with a `*.yuv.md5` list (`Executor.digest_by_frames`
/ `Executor.compare`, script/test/model/__init__.py:119-183).  This module does
the same on the planes the GPU path returns (`Decoder.deblock_filter`,
`DeviceBatch.planes`): 4:2:0, 8 bits per sample, frame coding -- the formats the
hot path reconstructs.

Host-side byte shuffling only (strided row copies); nothing here computes samples.
"""
from __future__ import annotations

import hashlib
import io
import os
from dataclasses import dataclass
from typing import BinaryIO, Iterable, Sequence

import numpy as np


@dataclass(frozen=True)
class Crop:
    """SPS frame cropping, in the syntax's units (output.cc:147-157): offsets count
    chroma samples horizontally and chroma rows x (2 - frame_mbs_only_flag) vertically."""
    left: int = 0
    right: int = 0
    top: int = 0
    bottom: int = 0
    frame_mbs_only: int = 1

    @staticmethod
    def for_height(width_mbs: int, height_mbs: int, width: int, height: int) -> "Crop":
        """The crop an encoder signals for a width x height picture coded in whole MBs
        (1920x1080 in 120x68 MBs -> frame_crop_bottom_offset 4)."""
        dx, dy = 16 * width_mbs - width, 16 * height_mbs - height
        if dx < 0 or dy < 0 or dx % 2 or dy % 2:
            raise ValueError(f"{width}x{height} does not fit {width_mbs}x{height_mbs} MBs in 4:2:0 crop units")
        return Crop(right=dx // 2, bottom=dy // 2)


@dataclass(frozen=True)
class OutputGeometry:
    """Cropped output sizes (output.cc:135-165)."""
    luma: tuple[int, int, int, int]      # (x0, y0, width, height) inside the coded luma plane
    chroma: tuple[int, int, int, int]
    fake_uv: int = 0                     # 4:0:0: bytes of value 128 per chroma plane (output.cc:205-224)

    @property
    def frame_bytes(self) -> int:
        """iFrameSize (output.cc:164): one byte per sample at 8 bits."""
        return self.luma[2] * self.luma[3] + 2 * self.chroma[2] * self.chroma[3] + 2 * self.fake_uv


def geometry(width_mbs: int, height_mbs: int, crop: Crop = Crop(), chroma_format: int = 1) -> OutputGeometry:
    """output.cc:135-165: size_x_l = PicWidthInMbs*16, size_x_c = PicWidthInMbs*MbWidthC;
    crop_*_c from the SPS (vertical offsets x (2 - frame_mbs_only_flag)), crop_*_l =
    SubWidthC/SubHeightC x crop_*_c.  chroma_format 2 (4:2:2): SubHeightC 1; 3 (4:4:4): SubWidthC 1 too;
    0 (4:0:0): the cropped luma, then two planes of 128 of a quarter of its size (WriteUV,
    output.cc:205-224: the reference fakes a 4:2:0 file)."""
    if chroma_format == 0:                   # CropUnitX 1, CropUnitY 2 - frame_mbs_only_flag (7.4.2.1.1)
        uy = 2 - crop.frame_mbs_only
        lw, lh = 16 * width_mbs - (crop.left + crop.right), 16 * height_mbs - uy * (crop.top + crop.bottom)
        if min(crop.left, crop.right, crop.top, crop.bottom) < 0 or lw <= 0 or lh <= 0:
            raise ValueError(f"frame cropping {crop} leaves no picture of {width_mbs}x{height_mbs} MBs")
        return OutputGeometry((crop.left, uy * crop.top, lw, lh), (0, 0, 0, 0), (lw * lh) // 4)
    sub_w, sub_h = (1 if chroma_format == 3 else 2), (2 if chroma_format == 1 else 1)
    lc, rc = crop.left, crop.right
    tc, bc = crop.top * (2 - crop.frame_mbs_only), crop.bottom * (2 - crop.frame_mbs_only)
    size_x_l, size_y_l = 16 * width_mbs, 16 * height_mbs
    size_x_c, size_y_c = 16 // sub_w * width_mbs, 16 // sub_h * height_mbs
    lw, lh = size_x_l - sub_w * (lc + rc), size_y_l - sub_h * (tc + bc)
    cw, ch = size_x_c - (lc + rc), size_y_c - (tc + bc)
    if min(lc, rc, tc, bc) < 0 or lw <= 0 or lh <= 0 or cw <= 0 or ch <= 0:
        raise ValueError(f"frame cropping {crop} leaves no picture of {width_mbs}x{height_mbs} MBs")
    return OutputGeometry((sub_w * lc, sub_h * tc, lw, lh), (lc, tc, cw, ch))


def _plane_view(p: np.ndarray, rect: tuple[int, int, int, int], name: str) -> np.ndarray:
    x0, y0, w, h = rect
    if p.dtype != np.uint8 or p.ndim != 2 or p.shape[0] < y0 + h or p.shape[1] < x0 + w:
        raise ValueError(f"{name} plane {p.dtype}{p.shape} does not hold the crop window {rect}")
    return p[y0:y0 + h, x0:x0 + w]


def frame_bytes(y: np.ndarray, u: np.ndarray, v: np.ndarray, geom: OutputGeometry) -> bytes:
    """One output frame as written by write_out_picture (output.cc:186-201): the cropped
    Y rows, then Cb, then Cr, each row-contiguous (img2buf, output.cc:61-106)."""
    out = bytearray(geom.frame_bytes)
    mv = memoryview(out)
    off = 0
    planes = ((y, geom.luma, "Y"),) if geom.fake_uv else ((y, geom.luma, "Y"), (u, geom.chroma, "Cb"), (v, geom.chroma, "Cr"))
    for p, rect, name in planes:
        view = _plane_view(np.asarray(p), rect, name)
        n = view.size
        mv[off:off + n] = np.ascontiguousarray(view).reshape(-1).data
        off += n
    if geom.fake_uv:
        mv[off:] = b"\x80" * (2 * geom.fake_uv)
    return bytes(out)


class YuvWriter:
    """Appends cropped frames to a file (or any binary stream), like the reference's
    output file descriptor `p_out` (output.cc:109, write() per plane)."""

    def __init__(self, target: str | os.PathLike | BinaryIO, width_mbs: int, height_mbs: int,
                 crop: Crop = Crop()):
        self.geom = geometry(width_mbs, height_mbs, crop)
        self._own = not hasattr(target, "write")
        self._f: BinaryIO = open(target, "wb") if self._own else target   # type: ignore[assignment]
        self.frames = 0

    def write(self, y: np.ndarray, u: np.ndarray, v: np.ndarray) -> None:
        data = frame_bytes(y, u, v, self.geom)
        if self._f.write(data) not in (None, len(data)):
            raise IOError("write_out_picture: error writing to YUV file")
        self.frames += 1

    def close(self) -> None:
        if self._own and not self._f.closed:
            self._f.close()

    def __enter__(self) -> "YuvWriter":
        return self

    def __exit__(self, *exc) -> None:
        self.close()


def digest_by_frames(source: str | os.PathLike | bytes, frames: int) -> list[str]:
    """Executor.digest_by_frames (model/__init__.py:119-150): split the decoded YUV into
    `frames` equal chunks (size // frames; a remainder becomes one more chunk) and MD5
    each, lower-case hex."""
    if frames <= 0:
        raise ValueError(f"digest error: {frames} frames")
    data = source if isinstance(source, (bytes, bytearray)) else open(source, "rb").read()
    size = len(data) // frames
    if size <= 0:
        raise ValueError(f"digest error: {len(data)} bytes for {frames} frames")
    f = io.BytesIO(data)
    lines = []
    while True:
        chunk = f.read(size)
        if not chunk:
            break
        lines.append(hashlib.md5(chunk).hexdigest().lower())
    return lines


def read_digests(path: str | os.PathLike) -> list[str]:
    """A `*.yuv.md5` list: one digest per line (model/__init__.py:157-159)."""
    with open(path, "rt") as f:
        return [line.rstrip().lower() for line in f]


def write_digests(path: str | os.PathLike, lines: Iterable[str]) -> None:
    with open(path, "wt") as f:
        for line in lines:
            f.write(f"{line}\n")


class CompareError(Exception):
    pass


def compare(lines: Sequence[str], hashes: Sequence[str], name: str = "") -> list[str]:
    """Executor.compare (model/__init__.py:152-183): the frame counts must agree, then
    every digest; the first mismatch raises with its index."""
    lines = [x.rstrip().lower() for x in lines]
    hashes = [x.rstrip().lower() for x in hashes]
    if len(lines) != len(hashes):
        raise CompareError(f"decoded frames is different: {name}")
    for i, (line, h) in enumerate(zip(lines, hashes)):
        if line != h:
            raise CompareError(f"mismatch {i} {name}: {line} != {h}")
    return lines


def compare_yuv(source: str | os.PathLike | bytes, digest_file: str | os.PathLike, name: str = "") -> list[str]:
    """The harness's compare() for a decoded file against its `*.yuv.md5`."""
    hashes = read_digests(digest_file)
    return compare(digest_by_frames(source, len(hashes)), hashes, name)
