"""Device-resident batches for h264r_decode_batch (throughput mode).

torch is used only as the device allocator (ROCm build: 'cuda' == HIP device);
the arrays are the canonical formats of include/h264r.h.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import _abi as A


@dataclass
class DeviceBatch:
    batch: A.Batch
    num_pics: int
    width_mbs: int
    height_mbs: int
    tensors: dict = field(default_factory=dict)   # keeps device memory alive
    chroma_format: int = 1

    def planes(self, i: int):
        """(Y, Cb, Cr) of picture i as numpy arrays (device -> host copy)."""
        W, H = self.width_mbs, self.height_mbs
        cw, ch = A.chroma_mb(self.chroma_format)
        y = self.tensors["out_y"][i].cpu().numpy().reshape(16 * H, 16 * W)
        u = self.tensors["out_u"][i].cpu().numpy().reshape(ch * H, cw * W)
        v = self.tensors["out_v"][i].cpu().numpy().reshape(ch * H, cw * W)
        return y, u, v


def pack(pictures, quant: np.ndarray):
    """Concatenate synth.Pictures into host arrays with one shared level pool."""
    W, H = pictures[0].cfg.width_mbs, pictures[0].cfg.height_mbs
    stride = max(len(p.slices) for p in pictures)
    mbs, lv, mv, rr, sl, pics = [], [], [], [], [], []
    off = 0
    for p in pictures:
        assert (p.cfg.width_mbs, p.cfg.height_mbs) == (W, H)
        m = p.mbs.copy()
        m["coef_off"] += off
        mbs.append(m)
        n = (len(p.levels) + 7) // 8 * 8
        l = np.zeros(n, np.int16)
        l[: len(p.levels)] = p.levels
        lv.append(l)
        off += n
        mv.append(p.mv)
        rr.append(p.ref_idx)
        s = np.zeros(stride, A.SLICE_DTYPE)
        s[: len(p.slices)] = p.slices
        sl.append(s)
        pics.append(p.pic)
    q = np.repeat(np.ascontiguousarray(quant, A.QUANT_DTYPE).reshape(1), len(pictures))
    return dict(mbs=np.concatenate(mbs), levels=np.concatenate(lv), mv=np.stack(mv), ref_idx=np.stack(rr),
                slices=np.concatenate(sl), pics=np.concatenate(pics), quant=q, stride=stride, W=W, H=H,
                chroma_format=A.idc_of(pictures[0].cfg.chroma_format))


def to_device(host: dict, n: int, ref_planes_ptr: int | None, device: str = "cuda") -> DeviceBatch:
    import torch

    def dev(a: np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(device)

    W, H = host["W"], host["H"]
    t = {k: dev(host[k]) for k in ("mbs", "levels", "mv", "ref_idx", "slices", "pics", "quant")}
    t["out_y"] = torch.zeros((n, 256 * W * H), dtype=torch.uint8, device=device)
    fmt = host.get("chroma_format", 1)
    cw, ch = A.chroma_mb(fmt)
    cs = cw * ch * W * H                                # 4:2:2 / 4:4:4: larger chroma planes
    t["out_u"] = torch.zeros((n, cs), dtype=torch.uint8, device=device)
    t["out_v"] = torch.zeros((n, cs), dtype=torch.uint8, device=device)
    b = A.Batch()
    b.num_pics, b.width_mbs, b.height_mbs, b.slice_stride = n, W, H, host["stride"]
    for k in ("mbs", "levels", "mv", "ref_idx", "slices", "pics", "quant", "out_y", "out_u", "out_v"):
        setattr(b, k, t[k].data_ptr())
    b.ref_planes = ref_planes_ptr
    # MBAFF frames take their own launch sequence (include/h264r.h h264r_batch.mbaff)
    b.mbaff = int(bool((host["pics"]["structure"] == A.MBAFF_FRAME).all()))
    return DeviceBatch(b, n, W, H, t, fmt)
