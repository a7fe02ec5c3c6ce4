"""N > 1 placement logic on CPU: gloo, world_size 2 (the GPU path uses the same code
with the nccl = RCCL backend)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from h264r import dist as D

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "arrow-h264_amd", "lib", "libh264r.so")


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_picture_share_disjoint():
    seen = []
    for r in range(4):
        seen += list(D.picture_share(r, 4, 8))
    assert sorted(seen) == list(range(32))
    with pytest.raises(ValueError):
        D.picture_share(4, 4, 8)


@pytest.mark.parametrize("starts,H,world,want", [
    ([0, 17, 34, 51], 68, 4, [(0, 17), (17, 34), (34, 51), (51, 68)]),        # config 4: 4 slices
    ([0, 17, 34, 51, 68, 85, 102, 118], 135, 8, None),                          # config 5: 8 slices
    ([0, 17, 34, 51], 68, 2, [(0, 34), (34, 68)]),
    ([0], 68, 2, [(0, 68), (68, 68)]),                                          # one slice: nothing to shard
])
def test_slice_bands(starts, H, world, want):
    bands = D.slice_bands(starts, H, world)
    assert len(bands) == world and bands[0][0] == 0 and bands[-1][1] == H
    assert all(a[1] == b[0] for a, b in zip(bands, bands[1:]))
    assert all(b0 in starts + [H] and b1 in starts + [H] for b0, b1 in bands)
    if want is not None:
        assert bands == want
    else:
        assert [b1 - b0 for b0, b1 in bands] == [17, 17, 17, 17, 17, 17, 16, 17]


@pytest.mark.parametrize("bands,span", [([(0, 17), (17, 34), (34, 51), (51, 68)], 17),
                                        ([(0, 34), (34, 67)], 34), ([(0, 34), (34, 68)], 34),
                                        ([(0, 17), (17, 35)], 0), ([(0, 20), (20, 34)], 20), ([(0, 10), (10, 30)], 0),
                                        ([(0, 68), (68, 68)], 68)])
def test_uniform_span(bands, span):
    assert D.uniform_span(bands) == span


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        W = 5                              # MB columns of a toy picture
        # the in-place exchange into a DPB slot: uniform bands (one chunk per rank lands
        # straight in the slot) and non-uniform ones (padded + copied)
        ok_slot = []
        for starts, Hs in (([0, 3], 5), ([0, 2, 3, 5], 6), ([0, 4], 7)):
            bands2 = D.slice_bands(starts, Hs, world)
            Wb = W * 16
            src = torch.zeros(Hs * 16 * Wb, dtype=torch.uint8)
            a0, a1 = bands2[rank]
            for y in range(a0 * 16, a1 * 16):
                src[y * Wb:(y + 1) * Wb] = (y * 7 + 1) % 251
            cap = D.slot_capacity(Hs * 16, Wb, bands2, 16) + 64
            dst = torch.full((cap,), 0xEE, dtype=torch.uint8)
            send = torch.zeros(max(b1 - b0 for b0, b1 in bands2) * 16 * Wb, dtype=torch.uint8)
            send[: (a1 - a0) * 16 * Wb] = src[a0 * 16 * Wb: a1 * 16 * Wb]
            D.allgather_into_slot(send, dst, bands2, rank, 16, Wb)
            exp = torch.tensor([(y * 7 + 1) % 251 for y in range(Hs * 16)], dtype=torch.uint8).repeat_interleave(Wb)
            ok_slot.append(bool(torch.equal(dst[: Hs * 16 * Wb], exp)) and bool((dst[-64:] == 0xEE).all()))
        t = D.max_over_ranks(1.0 + rank)
        share = list(D.picture_share(rank, world, 3))
        q.put((rank, all(ok_slot), t, share))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_allgather_and_max():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [True, True]
    assert [r[2] for r in res] == [2.0, 2.0]           # the slowest rank's time on every rank
    assert res[0][3] == [0, 1, 2] and res[1][3] == [3, 4, 5]


def test_halo_rows():
    # luma window rows y-2 .. y+6, y = Y + floor(mv_y / 4); chroma rows yc .. yc+2
    assert D.halo_mb_rows(0) == 1
    assert D.halo_mb_rows(4 * 13) == 1              # 13 + 3 = 16 rows
    assert D.halo_mb_rows(4 * 13 + 1) == 2
    assert D.halo_mb_rows(131) == 3                 # config 5: |mv_y| <= 32.75 px
    assert D.halo_plan([(0, 17), (17, 34), (34, 51)], 1, 3) == ({0: (14, 17), 2: (34, 37)}, {0: (17, 20), 2: (31, 34)})
    assert D.halo_plan([(0, 2), (2, 4), (4, 9)], 0, 3) == ({1: (2, 4), 2: (4, 5)}, {1: (0, 2), 2: (1, 2)})
    assert D.halo_plan([(0, 9), (9, 9)], 1, 3) == ({}, {})


def _band_worker(rank, world, port, q, impl):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ok = []
        W, H, nk, slack = 3, 7, 3, 64
        for starts in ([0, 2, 3, 5], [0, 1, 4, 6], [0, 3]):
            bands = D.slice_bands(starts, H, world)
            for mode, halo in (("halo", 1), ("halo", 2), ("allgather", 0)):
                psz = [c * W * H for c in D.ROW_BYTES_PER_MB_COL]
                rb = [c * W for c in D.ROW_BYTES_PER_MB_COL]

                def value(k, pl, row):          # a byte per (picture, plane, MB row, offset)
                    n = rb[pl]
                    return (torch.arange(n, dtype=torch.int64) * 3 + k * 101 + pl * 37 + row * 13) % 251
                planes = [torch.full((nk * psz[pl] + slack,), 0xEE, dtype=torch.uint8) for pl in range(3)]
                b0, b1 = bands[rank]
                for pl in range(3):
                    v = planes[pl][: nk * psz[pl]].view(nk, psz[pl])
                    for k in range(nk):
                        for r in range(b0, b1):
                            v[k, r * rb[pl]:(r + 1) * rb[pl]] = value(k, pl, r).to(torch.uint8)
                X = D.BandExchange(bands, rank, W, H, nk, mode, halo, "cpu", impl=impl)
                X.run(planes)
                lo, hi = (0, H) if mode == "allgather" else (max(b0 - halo, 0), min(b1 + halo, H))
                if b1 <= b0 and mode == "halo":
                    lo, hi = b0, b0
                good = True
                for pl in range(3):
                    v = planes[pl][: nk * psz[pl]].view(nk, psz[pl])
                    for k in range(nk):
                        for r in range(H):
                            seg = v[k, r * rb[pl]:(r + 1) * rb[pl]]
                            want = value(k, pl, r).to(torch.uint8) if lo <= r < hi else torch.full_like(seg, 0xEE)
                            good &= bool(torch.equal(seg, want))
                    good &= bool((planes[pl][nk * psz[pl]:] == 0xEE).all())
                ok.append(good)
        q.put((rank, all(ok)))
    finally:
        dist.destroy_process_group()


IMPLS = ["torch", pytest.param("abi", marks=pytest.mark.skipif(not os.path.exists(LIB), reason="libh264r.so not built"))]


@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("world", [2, 3])
def test_gloo_band_exchange(world, impl):
    """BandExchange in both implementations: torch.distributed calls, and the library's
    h264r_group (include/h264r_group.h) over its callback transport, host planes."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_band_worker, args=(r, world, port, q, impl)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [True] * world


def _band_worker_c5(rank, world, port, q, impl):
    """Config 5's real geometry: 2160p = 135 MB rows in 8 slices of
    17 / 16 rows (synth.c slice_of_row), one band per rank, halo 3 MB rows (|mv_y| <= 32.75 px,
    dist.halo_mb_rows(131)) -- six interior ranks with two peers each -- in both modes."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        W, H, nk, slack = 2, 135, 2, 64
        starts = [0, 17, 34, 51, 68, 85, 102, 118]
        bands = D.slice_bands(starts, H, world)
        ok = [len(bands) == world]
        for mode, halo in (("halo", D.halo_mb_rows(131)), ("allgather", 0)):
            psz = [c * W * H for c in D.ROW_BYTES_PER_MB_COL]
            rb = [c * W for c in D.ROW_BYTES_PER_MB_COL]
            planes = [torch.full((nk * psz[pl] + slack,), 0xEE, dtype=torch.uint8) for pl in range(3)]
            b0, b1 = bands[rank]
            rowval = [[[((torch.arange(rb[pl], dtype=torch.int64) * 5 + k * 71 + pl * 29 + r * 11) % 251).to(torch.uint8)
                        for r in range(H)] for pl in range(3)] for k in range(nk)]
            for pl in range(3):
                v = planes[pl][: nk * psz[pl]].view(nk, psz[pl])
                for k in range(nk):
                    for r in range(b0, b1):
                        v[k, r * rb[pl]:(r + 1) * rb[pl]] = rowval[k][pl][r]
            X = D.BandExchange(bands, rank, W, H, nk, mode, halo, "cpu", impl=impl)
            X.run(planes)
            lo, hi = (0, H) if mode == "allgather" else (max(b0 - halo, 0), min(b1 + halo, H))
            for pl in range(3):
                v = planes[pl][: nk * psz[pl]].view(nk, psz[pl])
                for k in range(nk):
                    for r in range(H):
                        seg = v[k, r * rb[pl]:(r + 1) * rb[pl]]
                        want = rowval[k][pl][r] if lo <= r < hi else torch.full_like(seg, 0xEE)
                        ok.append(bool(torch.equal(seg, want)))
                ok.append(bool((planes[pl][nk * psz[pl]:] == 0xEE).all()))
            if mode == "halo":
                need, give = D.halo_plan(bands, rank, halo)
                ok.append(len(set(need) | set(give)) == (1 if rank in (0, world - 1) else 2))
        q.put((rank, all(ok), bands[rank]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("impl", IMPLS)
def test_gloo_world8_config5_bands(impl):
    world, port = 8, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_band_worker_c5, args=(r, world, port, q, impl)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [True] * world
    assert [tuple(r[2]) for r in res] == [(0, 17), (17, 34), (34, 51), (51, 68), (68, 85), (85, 102), (102, 118), (118, 135)]


@pytest.mark.skipif(not os.path.exists(LIB), reason="libh264r.so not built")
def test_group_plan_matches_halo_plan():
    """h264r_group_plan (the C ABI's plan) == dist.halo_plan in halo mode, and the all-gather plan
    (every other nonempty band whole), over random slice layouts, world 1..9."""
    import random
    from h264r import group as G
    rnd = random.Random(5)
    for _ in range(300):
        world = rnd.randint(1, 9)
        H = rnd.randint(1, 40)
        starts = sorted({0} | {rnd.randrange(H) for _ in range(rnd.randint(0, 8))})
        bands = D.slice_bands(starts, H, world)
        halo = rnd.randint(0, 4)
        for rank in range(world):
            assert G.plan(bands, rank, "halo", halo) == D.halo_plan(bands, rank, halo)
            need, give = G.plan(bands, rank, "allgather")
            assert need == {r: b for r, b in enumerate(bands) if r != rank and b[1] > b[0]}
            b0, b1 = bands[rank]
            assert give == ({r: (b0, b1) for r in range(world) if r != rank} if b1 > b0 else {})
            # pairwise consistency: what rank sends to r is what r receives from rank
            for r in range(world):
                if r != rank:
                    assert G.plan(bands, r, "halo", halo)[0].get(rank) == G.plan(bands, rank, "halo", halo)[1].get(r)


@pytest.mark.skipif(not os.path.exists(LIB), reason="libh264r.so not built")
def test_group_argument_errors():
    import ctypes as C
    import h264r
    from h264r import group as G
    L = h264r.lib()
    with pytest.raises(h264r.H264RError):
        G.plan([(0, 4), (4, 8)], 2)                       # rank outside the world
    with pytest.raises(KeyError):
        G.plan([(0, 4), (4, 8)], 0, "ring")
    b = (C.c_int32 * 4)(0, 4, 4, 8)
    n = (C.c_int32 * 4)()
    assert L.h264r_group_plan(2, 0, b, 7, 1, n, n) == h264r.A.EINVAL
    assert L.h264r_group_plan(2, 0, b, 0, -1, n, n) == h264r.A.EINVAL
    assert L.h264r_group_exchange(None, 1, None, None, None, 0, 0, None) == h264r.A.EINVAL
    h = C.c_void_p()
    assert L.h264r_group_create_transport(C.byref(h), -1, 2, 0, None) == h264r.A.EINVAL
    assert L.h264r_group_create(C.byref(h), -1, 2, 0, bytes(128)) == h264r.A.EINVAL
    # a transport group before set_bands: the exchange is out of order
    g = G.Group(1, 0, -1, "torch")
    buf = (C.c_uint8 * 4096)()
    with pytest.raises(h264r.H264RError):
        g.exchange(1, C.addressof(buf), C.addressof(buf), C.addressof(buf), 256, 64)
    g.set_bands(1, 1, [(0, 1)], "halo", 1, 2)
    g.exchange(1, C.addressof(buf), C.addressof(buf), C.addressof(buf), 256, 64)   # world 1: nothing to move
    with pytest.raises(h264r.H264RError):
        g.set_bands(1, 1, [(0, 2)], "halo", 1, 2)         # a band below the picture
    g.close()
