"""ctypes binding of include/h264r_group.h: the exchange of slice bands between ranks.

`Group` is one rank's handle.  Transport "rccl": the library's own RCCL communicator (rank 0
makes the unique id, torch.distributed broadcasts it); transport "torch": the library's callback
transport driven by torch.distributed point-to-point operations on host buffers -- the gloo
rehearsal (CPU tests, several ranks on one GPU, which RCCL refuses).  Planes are device memory
(device >= 0) or host memory (device -1, callback transport only).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _check, lib

HALO, ALLGATHER = 0, 1
MODES = {"halo": HALO, "allgather": ALLGATHER}
ID_BYTES = 128


class Transport(C.Structure):
    _fields_ = [("user", C.c_void_p),
                ("start", C.CFUNCTYPE(C.c_int, C.c_void_p)),
                ("send", C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_size_t)),
                ("recv", C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_size_t)),
                ("finish", C.CFUNCTYPE(C.c_int, C.c_void_p))]


def bind(L) -> None:
    P, I, I64 = C.c_void_p, C.c_int, C.c_int64
    sig = {
        "h264r_group_unique_id": ([P], I),
        "h264r_group_create": ([C.POINTER(P), I, I, I, P], I),
        "h264r_group_create_transport": ([C.POINTER(P), I, I, I, C.POINTER(Transport)], I),
        "h264r_group_destroy": ([P], I),
        "h264r_group_plan": ([I, I, P, I, I, P, P], I),
        "h264r_group_set_bands": ([P, I, I, P, I, I, I], I),
        "h264r_group_exchange": ([P, I, P, P, P, I64, I64, P], I),
        "h264r_group_stats": ([P, C.POINTER(I64), C.POINTER(I64), C.POINTER(I64)], I),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes, f.restype = args, res


def _bands_array(bands) -> np.ndarray:
    return np.ascontiguousarray(np.array([[b0, b1] for b0, b1 in bands], np.int32).reshape(-1))


def plan(bands, rank: int, mode: str = "halo", halo: int = 0):
    """h264r_group_plan: ({peer: (row0, row1)} received, {peer: (row0, row1)} sent)."""
    b = _bands_array(bands)
    n = len(bands)
    need, give = np.zeros(2 * n, np.int32), np.zeros(2 * n, np.int32)
    _check("h264r_group_plan", lib().h264r_group_plan(n, rank, b.ctypes.data, MODES[mode], halo,
                                                       need.ctypes.data, give.ctypes.data))
    pick = lambda a: {r: (int(a[2 * r]), int(a[2 * r + 1])) for r in range(n) if a[2 * r + 1] > a[2 * r]}
    return pick(need), pick(give)


def unique_id() -> np.ndarray:
    """h264r_group_unique_id: a fresh RCCL unique id (raises when librccl cannot be loaded)."""
    uid = np.zeros(ID_BYTES, np.uint8)
    _check("h264r_group_unique_id", lib().h264r_group_unique_id(uid.ctypes.data))
    return uid


class _TorchTransport:
    """The callback transport over torch.distributed (host buffers; gloo)."""

    def __init__(self, group=None):
        self.group = group
        self.ops = []
        self.keep = []
        self.struct = Transport(None, Transport._fields_[1][1](self._start), Transport._fields_[2][1](self._send),
                                Transport._fields_[3][1](self._recv), Transport._fields_[4][1](self._finish))

    @staticmethod
    def _tensor(buf, n):
        import torch
        return torch.from_numpy(np.ctypeslib.as_array((C.c_uint8 * n).from_address(buf)))

    def _start(self, _user):
        self.ops, self.keep = [], []
        return 0

    def _post(self, fn, peer, buf, n):
        import torch.distributed as dist
        try:
            t = self._tensor(buf, n)
            self.keep.append(t)
            self.ops.append(dist.P2POp(fn, t, peer, self.group))
            return 0
        except Exception:                       # noqa: BLE001 -- reported to the library as a failure
            return 1

    def _send(self, _user, peer, buf, n):
        import torch.distributed as dist
        return self._post(dist.isend, peer, buf, n)

    def _recv(self, _user, peer, buf, n):
        import torch.distributed as dist
        return self._post(dist.irecv, peer, buf, n)

    def _finish(self, _user):
        import torch.distributed as dist
        try:
            if self.ops:
                for q in dist.batch_isend_irecv(self.ops):
                    q.wait()
            return 0
        except Exception:                       # noqa: BLE001
            return 1
        finally:
            self.ops, self.keep = [], []


class Group:
    """One rank of an h264r_group (include/h264r_group.h)."""

    def __init__(self, nranks: int, rank: int, device: int, transport: str = "rccl", pg=None):
        L = lib()
        self._L = L
        self._h = C.c_void_p()
        self._transport = None
        if transport == "rccl":
            import torch
            import torch.distributed as dist
            uid = unique_id() if rank == 0 else np.zeros(ID_BYTES, np.uint8)
            if nranks > 1:
                t = torch.from_numpy(uid).to(f"cuda:{device}")
                dist.broadcast(t, 0, group=pg)
                uid = t.cpu().numpy()
            _check("h264r_group_create", L.h264r_group_create(C.byref(self._h), device, nranks, rank, uid.ctypes.data))
        elif transport == "torch":
            self._transport = _TorchTransport(pg)
            _check("h264r_group_create_transport",
                   L.h264r_group_create_transport(C.byref(self._h), device, nranks, rank, C.byref(self._transport.struct)))
        else:
            raise ValueError(transport)
        self.nranks, self.rank, self.device, self.transport = nranks, rank, device, transport

    def set_bands(self, width_mbs: int, height_mbs: int, bands, mode: str, halo: int, max_pics: int) -> None:
        b = _bands_array(bands)
        _check("h264r_group_set_bands", self._L.h264r_group_set_bands(self._h, width_mbs, height_mbs, b.ctypes.data,
                                                                       MODES[mode], halo, max_pics))

    def exchange(self, num_pics: int, y: int, u: int, v: int, stride_y: int, stride_c: int, stream=None) -> None:
        """y / u / v: addresses of picture 0's planes (device or host); stream: a hipStream_t address."""
        _check("h264r_group_exchange", self._L.h264r_group_exchange(self._h, num_pics, y, u, v, stride_y, stride_c,
                                                                     stream))

    def stats(self) -> tuple[int, int, int]:
        s, r, t = C.c_int64(), C.c_int64(), C.c_int64()
        _check("h264r_group_stats", self._L.h264r_group_stats(self._h, C.byref(s), C.byref(r), C.byref(t)))
        return s.value, r.value, t.value

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.h264r_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:                       # noqa: BLE001
            pass
