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


def rccl_group_ok() -> bool:
    """Whether this process can make the library's RCCL group (librccl loads, ncclGetUniqueId
    works).  Checked on every rank, and agreed, before the collective group creation, so that a
    rank without RCCL cannot leave the others waiting in ncclCommInitRank."""
    try:
        from .group import unique_id
        unique_id()
        return True
    except Exception:                           # noqa: BLE001 -- any failure means "no"
        return False


def max_over_ranks(seconds: float, device=None) -> float:
    """The job's time: the slowest rank's (bench.py contract)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def min_over_ranks(value: float, device=None) -> float:
    """The smallest value over the ranks (a verification flag: 1.0 on a rank that passed)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return float(t.item())


# ------------------------------------------------------ chain mode over per-picture DPBs
# bench.py's chain mode: every picture of a batch carries its own
# DPB table (h264r_batch.ref_planes_stride), so one launch decodes the next picture of any
# number of chains; the decoded planes of step t ARE the chains' references of step t+1 (two
# output sets per group, alternating), and the exchange only has to bring in the rows of the
# other ranks' bands that this rank's motion compensation can reach.

ROW_BYTES_PER_MB_COL = (256, 64, 64)       # bytes of one MB row per MB column: Y, Cb, Cr


def halo_mb_rows(max_abs_mvy_qpel: int) -> int:
    """MB rows of a reference picture above / below a band that the band's motion
    compensation can read, for vertical motion vectors |mv_y| <= max_abs_mvy_qpel.
    Luma (get_block_luma, inter_prediction.cc:158-340): a 4x4 block at rows Y..Y+3 reads
    rows y-2 .. y+6 with y = Y + floor(mv_y / 4): ceil(m / 4) + 2 rows above the band,
    floor(m / 4) + 3 below.  Chroma (get_block_chroma :342-406, 4:2:0): rows yc .. yc+2 with
    yc = Yc + floor(mv_y / 8): at most ceil(m / 8) + 1 chroma rows = ceil(m / 4) + 2 luma rows.
    Rows past the picture edge are clamped (:185-186), i.e. read inside the picture."""
    m = max(0, int(max_abs_mvy_qpel))
    return -(-((m + 3) // 4 + 3) // 16)


def halo_plan(bands, rank: int, halo: int):
    """Rows this rank receives from / sends to each other rank in halo mode:
    (need {peer: (row0, row1)}, give {peer: (row0, row1)}), MB rows, empty ranges left out."""
    b0, b1 = bands[rank]
    need, give = {}, {}
    if b1 <= b0:
        return need, give
    for r, (r0, r1) in enumerate(bands):
        if r == rank or r1 <= r0:
            continue
        n0, n1 = max(b0 - halo, r0), min(b1 + halo, r1)
        if n1 > n0:
            need[r] = (n0, n1)
        g0, g1 = max(r0 - halo, b0), min(r1 + halo, b1)
        if g1 > g0:
            give[r] = (g0, g1)
    return need, give


class BandExchange:
    """The exchange step of chain mode for one group of `nk` pictures decoded as slice bands:
    after rank `rank` has decoded MB rows bands[rank] of every picture into a set of output
    planes (Y, Cb, Cr: flat tensors holding [nk][plane] + slack), bring in the rows of the
    other bands it will read as references of the next step:

    * mode "halo": the rows within `halo` MB rows of its band (halo_mb_rows), one send and
      one receive per neighbouring rank -- point-to-point over xGMI (batch_isend_irecv),
      every plane of all nk pictures packed into one buffer per peer;
    * mode "allgather": every other band whole, one all-gather of all nk pictures' bands
      (padded to the widest band).

    impl "abi" (default) runs the exchange in the library (include/h264r_group.h: pack kernel,
    RCCL ncclSend / ncclRecv on the decode stream, unpack kernel; over gloo the library's callback
    transport with torch.distributed operations on host buffers).  impl "torch" is the same
    exchange in torch.distributed calls (round 4), kept for comparison.  With gloo (CPU
    rehearsal) device tensors are staged through host memory."""

    def __init__(self, bands, rank: int, width_mbs: int, height_mbs: int, nk: int, mode: str, halo: int,
                 device, group=None, impl: str = "abi"):
        import torch
        import torch.distributed as dist
        self.bands, self.rank, self.nk, self.mode, self.group = list(bands), rank, nk, mode, group
        self.impl = impl
        self.W, self.H = width_mbs, height_mbs
        self.rb = [c * width_mbs for c in ROW_BYTES_PER_MB_COL]           # bytes per MB row, per plane
        self.mbrow = sum(self.rb)
        self.psz = [r * height_mbs for r in self.rb]                      # plane bytes
        self.world = len(self.bands)
        if mode not in ("halo", "allgather"):
            raise ValueError(mode)
        if mode == "halo":
            self.need, self.give = halo_plan(self.bands, rank, halo)
        else:
            self.need = {r: b for r, b in enumerate(self.bands) if r != rank and b[1] > b[0]}
            self.give = {r: self.bands[rank] for r in range(self.world) if r != rank}
        self.wide = max(b1 - b0 for b0, b1 in self.bands)
        self.device = device
        if impl == "abi":
            from .group import Group, plan
            # the library's plan (h264r_group_plan): in all-gather mode a rank with an empty band
            # sends nothing
            self.need, self.give = plan(self.bands, rank, mode, halo)
            dev = torch.device(device)
            gloo = dist.get_backend(group) == "gloo"
            self.grp = Group(self.world, rank, dev.index if dev.type == "cuda" else -1,
                             "torch" if gloo else "rccl", group)
            self.grp.set_bands(width_mbs, height_mbs, self.bands, mode, halo, nk)
            return
        if impl != "torch":
            raise ValueError(impl)

        def buf(rows):
            return torch.empty(nk * rows * self.mbrow, dtype=torch.uint8, device=device)
        if mode == "halo":
            self.sbuf = {r: buf(g1 - g0) for r, (g0, g1) in self.give.items()}
            self.rbuf = {r: buf(n1 - n0) for r, (n0, n1) in self.need.items()}
        else:
            self.sbuf = {0: buf(self.wide)}
            self.rbuf = {0: torch.empty(self.world * nk * self.wide * self.mbrow, dtype=torch.uint8, device=device)}

    def bytes_in(self) -> int:
        """Bytes this rank receives per exchange (the padding of the all-gather included)."""
        if self.impl == "abi":
            return self.nk * self.mbrow * sum(n1 - n0 for n0, n1 in self.need.values())
        return sum(t.numel() for t in self.rbuf.values()) - (self.sbuf[0].numel() if self.mode == "allgather" else 0)

    def _views(self, planes):
        return [planes[k].reshape(-1)[: self.nk * self.psz[k]].view(self.nk, self.psz[k]) for k in range(3)]

    def _pack(self, views, b, rows, r0, r1):
        """Rows [r0, r1) of every picture into buffer b ([nk][rows * mbrow], Y then Cb then Cr)."""
        bv = b.view(self.nk, rows * self.mbrow)
        o = 0
        for k in range(3):
            n = (r1 - r0) * self.rb[k]
            bv[:, o:o + n].copy_(views[k][:, r0 * self.rb[k]:r1 * self.rb[k]])
            o += rows * self.rb[k]

    def _unpack(self, views, b, rows, r0, r1):
        bv = b.view(self.nk, rows * self.mbrow)
        o = 0
        for k in range(3):
            n = (r1 - r0) * self.rb[k]
            views[k][:, r0 * self.rb[k]:r1 * self.rb[k]].copy_(bv[:, o:o + n])
            o += rows * self.rb[k]

    def run(self, planes) -> None:
        import torch.distributed as dist
        if self.world == 1 or not (dist.is_available() and dist.is_initialized()):
            return
        if self.impl == "abi":
            import torch
            stream = torch.cuda.current_stream(planes[0].device).cuda_stream if planes[0].is_cuda else None
            self.grp.exchange(self.nk, planes[0].data_ptr(), planes[1].data_ptr(), planes[2].data_ptr(),
                              self.psz[0], self.psz[1], stream)
            return
        views = self._views(planes)
        gloo = dist.get_backend(self.group) == "gloo" and self.device != "cpu" and str(self.device) != "cpu"
        if self.mode == "allgather":
            b0, b1 = self.bands[self.rank]
            self._pack(views, self.sbuf[0], self.wide, b0, b1)
            send, recv = self.sbuf[0], self.rbuf[0]
            if gloo:
                hs, hr = send.cpu(), recv.cpu()
                dist.all_gather_into_tensor(hr, hs, group=self.group)
                recv.copy_(hr)
            else:
                dist.all_gather_into_tensor(recv, send, group=self.group)
            per = self.nk * self.wide * self.mbrow
            for r, (n0, n1) in self.need.items():
                self._unpack(views, recv[r * per:(r + 1) * per], self.wide, n0, n1)
            return
        for r, (g0, g1) in self.give.items():
            self._pack(views, self.sbuf[r], g1 - g0, g0, g1)
        if gloo:
            hs = {r: t.cpu() for r, t in self.sbuf.items()}
            hr = {r: t.cpu() for r, t in self.rbuf.items()}
            ops = [dist.P2POp(dist.isend, hs[r], r, self.group) for r in sorted(hs)] + \
                  [dist.P2POp(dist.irecv, hr[r], r, self.group) for r in sorted(hr)]
        else:
            ops = [dist.P2POp(dist.isend, self.sbuf[r], r, self.group) for r in sorted(self.sbuf)] + \
                  [dist.P2POp(dist.irecv, self.rbuf[r], r, self.group) for r in sorted(self.rbuf)]
        if ops:
            for q in dist.batch_isend_irecv(ops):
                q.wait()
        for r, (n0, n1) in self.need.items():
            if gloo:
                self.rbuf[r].copy_(hr[r])
            self._unpack(views, self.rbuf[r], n1 - n0, n0, n1)
