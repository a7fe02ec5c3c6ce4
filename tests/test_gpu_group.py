"""The multi-GPU exchange of the C ABI (include/h264r_group.h) on the GPU.

* RCCL: a one-rank group made from h264r_group_unique_id (the box has one GPU, and RCCL refuses two
  ranks on one device), a plan and an exchange that has nothing to move -- the library finds and
  drives librccl.
* The device pack / unpack kernels (k_band_copy): two and three ranks on the one GPU over the
  library's callback transport (gloo through torch.distributed, device planes staged through
  pinned host buffers), every row of every plane of every picture checked: the rows of the plan
  arrive, nothing else is written, the slack after the planes is untouched.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gpu_group_rccl_one_rank():
    import ctypes as C
    import torch
    import h264r
    from h264r import group as G
    L = h264r.lib()
    torch.cuda.init()
    uid = np.zeros(128, np.uint8)
    assert L.h264r_group_unique_id(uid.ctypes.data) == 0
    assert uid.any()
    g = G.Group(1, 0, 0, "rccl")
    g.set_bands(4, 3, [(0, 3)], "halo", 1, 2)
    y = torch.zeros(2 * 256 * 12 + 64, dtype=torch.uint8, device="cuda")
    u = torch.zeros(2 * 64 * 12 + 64, dtype=torch.uint8, device="cuda")
    v = torch.zeros_like(u)
    g.exchange(2, y.data_ptr(), u.data_ptr(), v.data_ptr(), 256 * 12, 64 * 12,
               torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert g.stats() == (0, 0, 0)
    with pytest.raises(h264r.H264RError):           # more pictures than the plan's capacity
        g.exchange(3, y.data_ptr(), u.data_ptr(), v.data_ptr(), 256 * 12, 64 * 12, None)
    with pytest.raises(h264r.H264RError):           # device planes must be 8-byte aligned
        g.exchange(1, y.data_ptr() + 1, u.data_ptr(), v.data_ptr(), 256 * 12, 64 * 12, None)
    g.close()
    h = C.c_void_p()
    assert L.h264r_group_create(C.byref(h), 0, 2, 2, uid.ctypes.data) == h264r.A.EINVAL


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from h264r import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ok = []
        W, H, nk, slack = 5, 11, 3, 64
        psz = [c * W * H for c in D.ROW_BYTES_PER_MB_COL]
        rb = [c * W for c in D.ROW_BYTES_PER_MB_COL]
        for starts in ([0, 2, 5, 8], [0, 4, 6, 9], [0, 6]):
            bands = D.slice_bands(starts, H, world)
            for mode, halo in (("halo", 1), ("halo", 3), ("allgather", 0)):
                val = lambda k, pl, r: ((torch.arange(rb[pl], dtype=torch.int64) * 7 + k * 89 + pl * 31 + r * 17) % 251
                                        ).to(torch.uint8)
                host = [torch.full((nk * psz[pl] + slack,), 0xEE, dtype=torch.uint8) for pl in range(3)]
                b0, b1 = bands[rank]
                for pl in range(3):
                    hv = host[pl][: nk * psz[pl]].view(nk, psz[pl])
                    for k in range(nk):
                        for r in range(b0, b1):
                            hv[k, r * rb[pl]:(r + 1) * rb[pl]] = val(k, pl, r)
                planes = [h.to("cuda:0") for h in host]
                X = D.BandExchange(bands, rank, W, H, nk, mode, halo, "cuda:0", impl="abi")
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    X.run(planes)
                torch.cuda.current_stream().wait_stream(side)
                got = [p.cpu() for p in planes]
                lo, hi = (0, H) if mode == "allgather" else (max(b0 - halo, 0), min(b1 + halo, H))
                if b1 <= b0 and mode == "halo":
                    lo, hi = b0, b0
                for pl in range(3):
                    gv = got[pl][: nk * psz[pl]].view(nk, psz[pl])
                    for k in range(nk):
                        for r in range(H):
                            seg = gv[k, r * rb[pl]:(r + 1) * rb[pl]]
                            want = val(k, pl, r) if lo <= r < hi else torch.full_like(seg, 0xEE)
                            ok.append(bool(torch.equal(seg, want)))
                    ok.append(bool((got[pl][nk * psz[pl]:] == 0xEE).all()))
                sent, recvd, transfers = X.grp.stats()
                ok.append(recvd == X.bytes_in() and transfers == len(X.need) + len(X.give))
                X.grp.close()
        q.put((rank, all(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gpu_group_device_planes(world):
    import torch.multiprocessing as mp
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [True] * world
