"""N > 1 placement logic on CPU: gloo, world_size 2 (the GPU path uses the same code
with the nccl = RCCL backend)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from h264r import dist as D


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


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        H, W = 6, 5                        # MB rows / MB cols of a toy picture
        bands = D.slice_bands([0, 2, 3, 5], H, world)
        plane = torch.zeros((H * 16, W * 16), dtype=torch.uint8)
        r0, r1 = bands[rank]
        plane[r0 * 16:r1 * 16] = 10 + rank            # this rank's decoded band
        D.allgather_rows(plane, 16, bands, rank)
        want = torch.zeros_like(plane)
        for k, (b0, b1) in enumerate(bands):
            want[b0 * 16:b1 * 16] = 10 + k
        ok_rows = bool(torch.equal(plane, want))
        t = D.max_over_ranks(1.0 + rank)
        share = list(D.picture_share(rank, world, 3))
        q.put((rank, ok_rows, t, share))
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
