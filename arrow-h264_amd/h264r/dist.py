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


def uniform_span(bands: Sequence[tuple[int, int]]) -> int:
    """MB rows per rank if band k starts at k * span for every rank (only the last band
    may be shorter), else 0.  Equal slices (configs 4/5) give such bands; then the
    concatenation of every rank's span-row chunk IS the picture, and the exchange can
    all-gather straight into the DPB slot."""
    span = bands[0][1] - bands[0][0]
    if span <= 0:
        return 0
    for k, (b0, b1) in enumerate(bands):
        if b0 != min(k * span, bands[-1][1]) or b1 - b0 > span:
            return 0
    return span


def slot_capacity(rows: int, row_bytes: int, bands: Sequence[tuple[int, int]], rows_per_mb: int) -> int:
    """Bytes a DPB slot plane needs so that allgather_into_slot can land every rank's
    span-row chunk in place (a short last band still receives a full chunk)."""
    span = uniform_span(bands) or max(b1 - b0 for b0, b1 in bands)
    return max(rows, len(bands) * span * rows_per_mb) * row_bytes


def allgather_into_slot(send, dst, bands: Sequence[tuple[int, int]], rank: int, rows_per_mb: int, row_bytes: int,
                        group=None) -> None:
    """Exchange step of slice mode, one RCCL all-gather per plane.  `send` holds this
    rank's band of the decoded plane from offset 0 (rows of `row_bytes`; at least as many
    rows as the widest band); `dst` is the flat DPB-slot plane in which every rank
    receives the whole picture (sized by slot_capacity).  With uniform bands the
    collective writes the slot directly; otherwise each band is padded to the widest one
    and copied into place after the gather."""
    import torch
    import torch.distributed as dist
    world = len(bands)
    span = uniform_span(bands)
    if span:
        n = span * rows_per_mb * row_bytes
        dist.all_gather_into_tensor(dst[: world * n], send[:n], group=group)
        return
    wide = max(b1 - b0 for b0, b1 in bands) * rows_per_mb * row_bytes
    recv = torch.empty(world * wide, dtype=send.dtype, device=send.device)
    dist.all_gather_into_tensor(recv, send[:wide], group=group)
    for k, (b0, b1) in enumerate(bands):
        a0, a1 = b0 * rows_per_mb * row_bytes, b1 * rows_per_mb * row_bytes
        dst[a0:a1] = recv[k * wide: k * wide + (a1 - a0)]


def max_over_ranks(seconds: float, device=None) -> float:
    """The job's time: the slowest rank's (bench.py contract)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ------------------------------------------------------------------ dependent chains
# Slice mode over a real stream (bench.py --chain): every picture of a chain predicts from
# the chain's previous decoded picture, so each reference picture crosses the ranks once,
# before the next picture of its chain may start -- the exchange is on the dependency
# path (slice walk slice_data.cc:640-650, idc 2 stopping the filter at slice edges
# deblock.cc:247-253).  K chains advance together: their pictures form one batch, chain k
# predicting from DPB slot k, and one all-gather per plane moves every rank's band of all
# K pictures at once.

def chain_slots(slices, chain: int, nchains: int):
    """Slice tables of a chain's picture: reference slot 0 (the picture's first list-0
    reference) becomes the chain's own slot `chain`, slot s >= 1 the shared static slot
    nchains + s - 1; unused entries (-1) stay."""
    import numpy as np
    out = slices.copy()
    rs = out["ref_slot"]
    rs[...] = np.where(rs == 0, chain, np.where(rs > 0, nchains + rs.astype(np.int16) - 1, rs)).astype(np.int8)
    if nchains + int(slices["ref_slot"].max()) - 1 >= 32:
        raise ValueError("chain slots exceed the 32 DPB slots of a batch")
    return out


def chain_exchange(out, slots, bands: Sequence[tuple[int, int]], rank: int, plane_bytes: int, slot_stride: int,
                   rows_per_mb: int, row_bytes: int, group=None) -> None:
    """Exchange of one plane in chain mode: `out` holds the K decoded planes of this rank
    ([K][plane_bytes], only this rank's band rows valid); `slots` the K chains' DPB slot
    planes ([K][slot_stride]).  Every rank's band of all K pictures travels in ONE
    all-gather (bands padded to the widest); each rank then lands every band in every
    chain's slot.  World 1: a local copy."""
    import torch
    import torch.distributed as dist
    world = len(bands)
    K = out.numel() // plane_bytes
    rb = rows_per_mb * row_bytes
    src = out.reshape(-1)[:K * plane_bytes].view(K, plane_bytes)
    dst = slots.reshape(-1)[:K * slot_stride].view(K, slot_stride)
    if world == 1 or not (dist.is_available() and dist.is_initialized()):
        dst[:, :plane_bytes].copy_(src)
        return
    wide = max(b1 - b0 for b0, b1 in bands) * rb
    a0, a1 = bands[rank][0] * rb, bands[rank][1] * rb
    send = torch.zeros((K, wide), dtype=out.dtype, device=out.device)
    if a1 > a0:
        send[:, :a1 - a0].copy_(src[:, a0:a1])
    recv = torch.empty((world, K, wide), dtype=out.dtype, device=out.device)
    dist.all_gather_into_tensor(recv.view(-1), send.view(-1), group=group)
    for r, (b0, b1) in enumerate(bands):
        if b1 > b0:
            dst[:, b0 * rb:b1 * rb].copy_(recv[r, :, :(b1 - b0) * rb])
