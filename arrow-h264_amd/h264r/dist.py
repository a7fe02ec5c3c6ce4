"""Multi-GPU placement of the reconstruction path: one process per GPU over
torch.distributed (backend "nccl" = RCCL on ROCm; "gloo" for the CPU tests).

SURVEY.md section 8(e):

* disable_deblocking_filter_idc 0 (config 3) chains every MB of a picture through the
  loop filter (deblock.cc:547-551), so a picture cannot be split: ranks are
  *replicas*, each decoding its own pictures -- no collective on the data path.
* idc 1/2 with several slices (configs 4/5): slices never predict across each other
  (intra_prediction.cc:145-152, interpret_mv.cc:35-38) and idc 2 stops the filter at
  slice edges (deblock.cc:247-253), so a picture shards into slice bands.  Every GPU
  then needs the whole decoded picture as a motion-compensation reference: one
  exchange per reference picture, an all-gather of the finished bands.
"""
from __future__ import annotations

from typing import Sequence


def picture_share(rank: int, world: int, n_per_rank: int) -> range:
    """Replica mode: the picture indices rank `rank` decodes (disjoint across ranks)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    return range(rank * n_per_rank, (rank + 1) * n_per_rank)


def slice_bands(slice_first_rows: Sequence[int], height_mbs: int, world: int) -> list[tuple[int, int]]:
    """Slice mode: split a picture whose slices start at the given MB rows into `world`
    contiguous bands of whole slices, balanced by MB rows.  Returns [(row0, row1)] per
    rank (possibly empty bands when there are fewer slices than ranks)."""
    starts = sorted(set(int(r) for r in slice_first_rows))
    if not starts or starts[0] != 0 or starts[-1] >= height_mbs:
        raise ValueError("slices must start at row 0 and inside the picture")
    bounds = starts + [height_mbs]
    cuts = [0]
    for k in range(1, world):
        target = height_mbs * k / world
        cand = [b for b in bounds if b >= cuts[-1]]
        cuts.append(min(cand, key=lambda b: (abs(b - target), -b)))
    cuts.append(height_mbs)
    return [(cuts[k], cuts[k + 1]) for k in range(world)]


def allgather_rows(plane, rows_per_mb: int, bands: Sequence[tuple[int, int]], rank: int, group=None):
    """Exchange step of slice mode: every rank holds the rows of its own band of `plane`
    (a [H, W] tensor, filled in place); after the call every rank holds the full plane.
    One all-gather of equal-sized (padded) bands; on ROCm with the nccl backend this is
    RCCL over xGMI."""
    import torch
    import torch.distributed as dist
    H, W = plane.shape
    world = len(bands)
    span = max(b1 - b0 for b0, b1 in bands) * rows_per_mb
    if span == 0:
        return plane
    send = torch.zeros((span, W), dtype=plane.dtype, device=plane.device)
    r0, r1 = bands[rank][0] * rows_per_mb, bands[rank][1] * rows_per_mb
    send[: r1 - r0] = plane[r0:r1]
    recv = [torch.empty_like(send) for _ in range(world)]
    dist.all_gather(recv, send, group=group)
    for k, (b0, b1) in enumerate(bands):
        a0, a1 = b0 * rows_per_mb, b1 * rows_per_mb
        plane[a0:a1] = recv[k][: a1 - a0]
    return plane


def max_over_ranks(seconds: float, device=None) -> float:
    """The job's time: the slowest rank's (bench.py contract)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
