#!/usr/bin/env python3
"""Benchmark: macroblocks/s of post-entropy reconstruction (MC + IDCT + intra +
deblock) on MI355X, BASELINE.json's metric.

One GPU (default): throughput mode, the headline.  A step = one h264r_decode_batch over a
batch of synthetic pictures already resident in HBM (B independent pictures
sharing a reference set).  Workload: SURVEY config 3, 1080p (120x68 MBs) IPPP Main P
pictures, B = 1024 per GPU (the order-dependent walks need many pictures in flight).

N > 1 GPUs (default): the headline workload as N replicas (config 3 pictures, B per rank, no
collective: disable_deblocking_filter_idc 0 chains every MB of a picture through the loop filter,
deblock.cc:547-551), value = all ranks' MBs / the slowest rank's time -- the same workload as the
one-GPU line, so the scaling curve compares like with like.  Beside it in the same line,
`slice_sharded`: chain mode on config 5 (2160p High B pictures, 8 slices,
disable_deblocking_filter_idc 2), K = 32 x N dependent chains advance one picture per step, each
rank decodes its band of slices of every picture, and the rows of the other bands that its next
motion compensation can reach come in by point-to-point RCCL transfers over xGMI (or --exchange
allgather: every band); weak scaling, with the one-GPU line of the same mode (`same_mode_n1`)
and its CPU baseline.  `--mode chain` makes the chain line the whole output.  `--gpus N`
without a launcher starts the N ranks itself (torch.distributed.run as a child process); under
`torch.distributed.run` one process per GPU reads RANK / LOCAL_RANK / WORLD_SIZE.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "arrow-h264_amd"))

import numpy as np  # noqa: E402

CONFIG_NAMES = {2: "1080p all-intra", 3: "1080p IPPP Main P-frames", 4: "1080p High IBBP B-frames, 4 slices",
                5: "2160p High B-frames, 8 slices"}
CONFIG_SIZE = {2: (120, 68), 3: (120, 68), 4: (120, 68), 5: (240, 135)}
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_ISSUE_PER_S = 256 * 4 * 2.4e9 / 2   # wave64 VALU instructions per second: 256 CUs x 4 SIMD-32 at 2.4 GHz, 2 cycles each


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(cfg, refs, seconds: float):
    """Oracle restatement (CPU port of the reference path), 1 thread, on a bounded
    sample of the same workload: pictures are generated first, only decode is timed."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    from h264r import synth
    from h264r import dist as D
    L = O.lib()
    nmb = cfg.width_mbs * cfg.height_mbs
    t0 = time.perf_counter()
    O.decode(synth.picture(L, cfg, 10_000), refs)
    per_pic = max(time.perf_counter() - t0, 1e-3)
    n = max(1, int(seconds / per_pic))
    pics = [synth.picture(L, cfg, 10_001 + i) for i in range(n)]
    t0 = time.perf_counter()
    for p in pics:
        O.decode(p, refs)
    el = time.perf_counter() - t0
    return n * nmb, el, n


def cpu_baseline_threads(cfg, refs, seconds: float, threads: int):
    """The same oracle with `threads` pthreads over independent pictures
    (oracle_decode_pictures; BASELINE.md section 4, 'nproc threads'), bounded sample."""
    import ctypes as C
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    from h264r import synth
    L = O.lib()
    W, H = cfg.width_mbs, cfg.height_mbs
    q = O.quant_flat()
    keep = []

    def batch(first, count):
        arr = (O.OraclePicture * count)()
        for i in range(count):
            p = synth.picture(L, cfg, first + i)
            out = O.new_planes(W, H)
            keep.append((p, out))
            arr[i] = O.make_oracle_picture(p, refs, q, out)
        return arr
    probe = batch(20_000, threads)
    t0 = time.perf_counter()
    L.oracle_decode_pictures(probe, threads, threads)
    per_round = max(time.perf_counter() - t0, 1e-3)
    n = threads * max(1, int(seconds / per_round))
    arr = batch(20_000 + threads, n)
    t0 = time.perf_counter()
    st = L.oracle_decode_pictures(arr, n, threads)
    el = time.perf_counter() - t0
    if st != 0:
        raise RuntimeError(f"oracle_decode_pictures -> {st}")
    return n * W * H, el, n


def kernel_bytes(pics, nmb):
    """The path's algorithmic bytes (R + W per MB, summed over the batch) split
    over the kernels without double counting: an MB's R (record, levels, motion, reference
    samples) to the kernel that reconstructs it (inter / PCM MBs k_inter4, intra MBs the
    intra kernels), every MB's W (384 final samples) to the deblocking kernel that stores
    them.  The three parts add up to the path's bytes; the unfiltered samples the
    reconstruction kernels write and the deblocking kernel reads back are not algorithmic
    (a fused design keeps them on chip), so they appear only in the PMC traffic."""
    from h264r import _abi as A
    inter = intra = 0
    pop4 = np.array([bin(v).count("1") for v in range(16)])
    for p in pics:
        m = p.mbs
        cbp = m["cbp"].astype(np.int64)
        cbpl, cbpc = cbp & 15, cbp >> 4
        typ = m["mb_type"]
        is_intra = (m["flags"] & A.MBF_INTRA) != 0
        pcm = typ == A.I_PCM
        i16 = typ == A.I_16x16
        Wm, Hm = p.cfg.width_mbs, p.cfg.height_mbs
        used = (p.ref_idx.reshape(2, Hm, 4, Wm, 4) >= 0).any(axis=(2, 4)).reshape(2, -1)
        nl = used.sum(axis=0)
        r = 32 + 128 * pop4[cbpl] + 32 * i16 + 16 * (cbpc != 0) + 256 * (cbpc == 2) + 464 * np.where(is_intra, 0, nl)
        r = np.where(pcm, 416, r)
        intra += int(r[is_intra & ~pcm].sum())
        inter += int(r[~is_intra | pcm].sum())
    return [inter, intra, len(pics) * nmb * 384]


def latency_chain(dec, L, cfg, refs, stream, n: int, verify: int):
    """SURVEY 8(d) latency mode: a dependent IPPP chain decoded one picture per launch.
    Picture i predicts from DPB slot 0 = the decoded picture i-1 (slot 1 keeps the
    synthetic reference), so every launch waits for the previous one's output.  Returns
    (ms per picture, pictures, verified): the first `verify` pictures are compared with
    the oracle's chain."""
    import torch
    import h264r
    from h264r import batch as B
    from h264r import synth
    W, H = cfg.width_mbs, cfg.height_mbs
    slack = 64
    sizes = (256 * W * H, 64 * W * H, 64 * W * H)

    def planes_t(src=None):
        if src is None:
            return [torch.zeros(n_ + slack, dtype=torch.uint8, device="cuda") for n_ in sizes]
        return [torch.from_numpy(np.concatenate([a.reshape(-1), np.zeros(slack, np.uint8)])).to("cuda") for a in src]
    bufs = [planes_t(refs[0]) if refs else planes_t()] + [planes_t() for _ in range(n)]
    slot1 = [planes_t(r) for r in refs[1:]]
    pics = [synth.picture(L, cfg, 50_000 + i) for i in range(n)]
    keep, batches = [], []
    for i, p in enumerate(pics):
        tab = np.zeros(3 * 32, np.int64)
        for s_, planes in enumerate([bufs[i]] + slot1):
            for k in range(3):
                tab[3 * s_ + k] = planes[k].data_ptr()
        tab_t = torch.from_numpy(tab).to("cuda")
        db = B.to_device(B.pack([p], h264r.quant_flat()), 1, tab_t.data_ptr())
        db.batch.out_y, db.batch.out_u, db.batch.out_v = (t.data_ptr() for t in bufs[i + 1])
        keep.append((tab_t, db))
        batches.append(db.batch)

    def chain():
        for b in batches:
            dec.decode_batch(b, stream)
    chain()                                            # warm-up (and the verified run)
    torch.cuda.synchronize()
    dec.check()
    verified = None
    if verify:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import _oracle as O
        oref = list(refs)
        verified = True
        for i in range(min(verify, n)):
            want = O.decode(pics[i], oref)
            got = [bufs[i + 1][k][: sizes[k]].cpu().numpy() for k in range(3)]
            verified &= all(np.array_equal(got[k], want[k].reshape(-1)) for k in range(3))
            oref = [want] + oref[1:] if refs else []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    chain()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3, n, verified


class GpuTurn:
    """Rehearsal only (H264R_BENCH_REHEARSE=1: several ranks on one GPU): one rank's decode on the
    device at a time.  Two processes' launch sequences side by side on one GPU can starve each
    other's k_intra_levels, whose grid barrier needs the whole grid resident; the bounded wait
    then expires and h264r_check reports H264R_EDEVICE.  A file lock held from the launch until
    the device has drained keeps the decodes apart (the exchange still runs concurrently).  On
    separate GPUs (the real N > 1 run) this is a no-op."""

    def __init__(self, on: bool):
        self.fd = None
        if on:
            self.fd = open(f"/tmp/h264r_rehearse_{os.environ.get('MASTER_PORT', '0')}.lock", "w")

    def __enter__(self):
        if self.fd is not None:
            import fcntl
            fcntl.flock(self.fd, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        if self.fd is not None:
            import fcntl
            import torch
            torch.cuda.synchronize()
            fcntl.flock(self.fd, fcntl.LOCK_UN)
        return False


def chain_run(args, rank: int, world: int, local: int, cs, rehearse: bool, nchains: int, cfg_idx: int,
              exchange: str) -> dict:
    """Dependent chains, slice-sharded.  `nchains` chains advance
    one picture per step; chain k's picture t predicts from its own picture t-1, so every decoded
    picture is a reference the next step needs on every rank that reads it.

    * Every picture of a batch has its own DPB table (h264r_batch.ref_planes_stride): slot 0 =
      its chain's previous picture, slots 1.. = static references shared by all chains.  The
      chains form `--chain-groups` groups (default 1), one launch each per step.
    * A group keeps two output sets; step t decodes into set t % 2 and reads set (t+1) % 2 -- the
      previous step's output IS the reference, nothing is copied on a rank.
    * Each rank decodes its slice band (MB rows of whole slices, disable_deblocking_filter_idc 2:
      deblock.cc:247-253; slices never predict across each other: intra_prediction.cc:145-152),
      then the exchange brings in the rows of other bands its next motion compensation can reach:
      `halo` (default) = the rows within halo_mb_rows(max |mv_y|) of its band from the
      neighbouring ranks, point-to-point (RCCL send/recv over xGMI); `allgather` = every band of
      every picture (one all-gather per group and step).  With two or more groups the exchange of
      one group (communication stream) overlaps the decode of the next (decode stream); each is
      on its chains' dependency path.  One group (the default) decodes all chains in one launch:
      the deblocking walks, latency-bound at these batch sizes, then run side by side, which
      outweighs hiding an exchange of a few MB rows.  The slice walk this parallelises is
      slice_data.cc:640-650."""
    import torch
    import h264r
    from h264r import batch as B
    from h264r import synth
    from h264r import dist as D
    L = h264r.lib()
    W, H = CONFIG_SIZE[cfg_idx]
    cfg = synth.default_cfg(L, cfg_idx, W, H)
    refs = synth.refpics(L, cfg)
    if not refs:
        raise SystemExit("chain mode needs inter pictures (configs 3, 4, 5)")
    ng = max(1, int(getattr(args, "chain_groups", 1) or 1))
    if nchains < ng or nchains % ng:
        raise SystemExit(f"chain mode takes a multiple of --chain-groups ({ng}) chains")
    nk = nchains // ng
    nmb = W * H
    # distinct synthetic pictures: up to 16 per group (chains beyond reuse them; every chain
    # still decodes its own picture from its own reference every step)
    nbase = min(nk, 16)
    base = [[synth.picture(L, cfg, g * 1000 + i) for i in range(nbase)] for g in range(ng)]
    srow = base[0][0].mbs["slice"].reshape(H, W)[:, 0]
    first = [0] + [r for r in range(1, H) if srow[r] != srow[r - 1]]
    bands = D.slice_bands(first, H, world) if world > 1 else [(0, H)]
    band = bands[rank]
    if world > 1 and cfg.deblock_idc == 0:
        raise SystemExit("slice sharding needs disable_deblocking_filter_idc 1/2 (configs 4, 5)")
    # the halo: every vertical motion vector of every picture (a decoder knows its next
    # picture's vectors before reconstructing it: the parser runs ahead of the GPU)
    mvy = max(int(np.abs((p.mv >> 16).astype(np.int16)).max()) for g in base for p in g)
    halo = D.halo_mb_rows(mvy)
    slack = 64
    psz = (256 * nmb, 64 * nmb, 64 * nmb)
    # the exchange: the library's (include/h264r_group.h) unless --exchange-impl torch; over RCCL
    # every rank first checks that it can load librccl, and the ranks agree, before the
    # collective group creation (a rank without it would leave the others waiting)
    impl, impl_note = getattr(args, "exchange_impl", "abi"), None
    if world > 1 and impl == "abi" and not rehearse:
        if D.min_over_ranks(1.0 if D.rccl_group_ok() else 0.0, device="cuda") < 1.0:
            impl, impl_note = "torch", "librccl not loadable on every rank: torch.distributed exchange"
    dec = h264r.Decoder(local, W, H)
    static = [[torch.from_numpy(np.concatenate([a.reshape(-1), np.zeros(slack, np.uint8)])).to("cuda") for a in r]
              for r in refs[1:]]
    groups = []
    for g in range(ng):
        pics = [base[g][k % nbase] for k in range(nk)]
        # two output sets [nk][plane] + slack; set 1 starts as every chain's first reference
        sets = [[torch.zeros(nk * psz[k3] + slack, dtype=torch.uint8, device="cuda") for k3 in range(3)]
                for _ in range(2)]
        for k3 in range(3):
            sets[1][k3][: nk * psz[k3]].view(nk, psz[k3]).copy_(
                torch.from_numpy(refs[0][k3].reshape(1, -1)).expand(nk, -1))
        tabs = []
        for si in range(2):                        # the table of a step that READS set si
            tab = np.zeros((nk, 3 * 32), np.int64)
            for k in range(nk):
                for k3 in range(3):
                    tab[k, k3] = sets[si][k3].data_ptr() + k * psz[k3]
                for j, planes in enumerate(static):
                    for k3 in range(3):
                        tab[k, 3 * (1 + j) + k3] = planes[k3].data_ptr()
            tabs.append(torch.from_numpy(tab.reshape(-1)).to("cuda"))
        db = B.to_device(B.pack(pics, h264r.quant_flat()), nk, tabs[1].data_ptr())
        db.batch.ref_planes_stride = 3 * 32
        for t_ in ("out_y", "out_u", "out_v"):          # the sets replace the batch's own outputs
            del db.tensors[t_]
        xch = D.BandExchange(bands, rank, W, H, nk, exchange, halo, f"cuda:{local}", impl=impl) if world > 1 else None
        groups.append(dict(pics=pics, sets=sets, tabs=tabs, db=db, xch=xch, ev_ex=[]))
    comm = torch.cuda.Stream(device=local) if world > 1 else None
    stream = cs.cuda_stream
    nstep = [0]
    turn = GpuTurn(rehearse and world > 1)

    def step():
        t = nstep[0]
        nstep[0] += 1
        for G in groups:
            if t >= 1 and comm is not None:
                cs.wait_event(G["ev_ex"][t - 1])       # the references of this step are complete
            wr, rd_ = G["sets"][t % 2], t % 2 ^ 1
            b = G["db"].batch
            b.out_y, b.out_u, b.out_v = (x.data_ptr() for x in wr)
            b.ref_planes = G["tabs"][rd_].data_ptr()
            if band[1] > band[0]:
                with turn:
                    dec.decode_batch(b, stream, rows=None if band == (0, H) else band)
            if comm is None:
                continue
            ev = torch.cuda.Event()
            ev.record(cs)
            comm.wait_event(ev)
            with torch.cuda.stream(comm):
                G["xch"].run(wr)
                ex = torch.cuda.Event()
                ex.record(comm)
            G["ev_ex"].append(ex)

    verified = None
    if not args.no_verify:
        # two steps, then chain 0 of group 0 against the oracle's chain: its second picture read
        # the first one through the exchange, so the band (and the halo rows received) must equal
        # the oracle's whole-picture decode
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import _oracle as O
        step()
        step()
        torch.cuda.synchronize()
        dec.check()
        rows = (16, 8, 8)
        ok = True
        # chain 0 of the first group and the last chain of the last group (its pictures sit at
        # the far end of the batch and read their own DPB table: ref_planes_stride)
        for G, k in ((groups[0], 0), (groups[-1], nk - 1)):
            want0 = O.decode(G["pics"][k], refs)
            want1 = O.decode(G["pics"][k], [want0] + list(refs[1:]))
            for t, want, lo, hi in ((0, want0, max(band[0] - halo, 0), min(band[1] + halo, H)), (1, want1, band[0], band[1])):
                if exchange == "allgather" and t == 0:
                    lo, hi = 0, H
                if hi <= lo:
                    continue
                for k3 in range(3):
                    got = G["sets"][t][k3][k * psz[k3]: (k + 1) * psz[k3]].cpu().numpy().reshape(want[k3].shape)
                    ok &= bool(np.array_equal(got[lo * rows[k3]:hi * rows[k3]], want[k3][lo * rows[k3]:hi * rows[k3]]))
        verified = bool(ok) if world == 1 else \
            bool(D.min_over_ranks(1.0 if ok else 0.0, device="cpu" if rehearse else "cuda") == 1.0)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    dec.set_timing(True)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    dec.check()
    kern = np.array(dec.last_timing()) * ng if band[1] > band[0] else np.zeros(4)  # ng launches per step
    dec.set_timing(False)
    if world > 1:
        dt = D.max_over_ranks(dt, device="cpu" if rehearse else "cuda")
    rd = wr = 0
    for g in range(ng):
        for k in range(nk):
            r, w = synth.algo_bytes(L, base[g][k % nbase])
            rd, wr = rd + r, wr + w
    total_mbs = nchains * nmb * args.steps
    value = total_mbs / dt
    frac_rows = (band[1] - band[0]) / H
    step_bytes = int((rd + wr) * frac_rows)
    achieved = step_bytes / (kern[3] * 1e-3) / 1e9 if kern[3] > 0 else 0.0
    xin = groups[0]["xch"].bytes_in() * ng if world > 1 else 0
    xops = 0 if world == 1 else ng * xch_ops(groups[0]["xch"], bands, rank, halo, exchange)
    del groups, dec
    torch.cuda.empty_cache()
    # PMC traffic of this mode (tools/pmc.sh over a chain-mode run -> profiles/traffic_c<N>_chain.json)
    traffic, traffic_src = None, None
    tpath = os.path.join(ROOT, "profiles", f"traffic_c{cfg_idx}_chain.json")
    if os.path.exists(tpath):
        tj = json.load(open(tpath))
        if tj.get("survey_config") == cfg_idx:
            per_mb = sum(v["traffic_bytes_per_mb"] for v in tj["kernels"].values())
            traffic = int(per_mb * nchains * nmb * frac_rows)   # this rank's band of every chain
            traffic_src = f"{os.path.basename(tpath)} ({tj.get('source')}): all kernels of the sequence"
    # the CPU path beside it (rank 0 at one GPU): the oracle port on a bounded sample of the same
    # pictures, 1 thread and a thread pool (a chain's picture costs the CPU what an independent one does)
    cpu = cpu_mt = None
    if world == 1 and not args.no_cpu:
        done, el, ncpu = cpu_baseline(cfg, refs, args.cpu_seconds)
        cpu = {"value": done / el, "unit": "macroblocks/s", "cores": 1, "kind": "port",
               "sample": f"{ncpu} pictures of {CONFIG_NAMES[cfg_idx]} ({ncpu * nmb} MBs, {el:.1f} s) decoded by "
                         f"oracle/h264r_oracle.c (1 thread) on {cpu_model()}"}
        thr = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        done, el, ncpu = cpu_baseline_threads(cfg, refs, args.cpu_seconds / 2, thr)
        cpu_mt = {"value": done / el, "unit": "macroblocks/s", "cores": thr, "kind": "port",
                  "sample": f"{ncpu} pictures ({ncpu * nmb} MBs, {el:.1f} s) over {thr} threads, "
                            f"oracle_decode_pictures, on {cpu_model()}"}
    return {
        "metric": f"macroblocks/s (decode reconstruct, post-entropy) {CONFIG_NAMES[cfg_idx]}, dependent chains"
                  f"{', slice-sharded' if world > 1 else ''}; % HBM roofline",
        "value": value, "unit": "macroblocks/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic (seeded SURVEY 8(d) generator, arrow-h264_amd/csrc/synth.c)",
        "config": {"workload": f"{CONFIG_NAMES[cfg_idx]}, {nchains} dependent chains ({nchains // world} per GPU; "
                               "each picture predicts from its chain's previous decoded picture)",
                   "survey_config": cfg_idx, "width_mbs": W, "height_mbs": H, "mode": "chain",
                   "chains": nchains, "chains_per_gpu": nchains // world, "chain_groups": ng,
                   "parallelism": f"slices{world}" if world > 1 else "single",
                   "rows_this_rank": list(band), "bands": [list(b) for b in bands]},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "h264r_decode_batch launch sequences of the chain groups (one per group)",
                     "kernel_ms": float(kern[3]), "kernel_algo_bytes": step_bytes,
                     "numerator": "SURVEY 8(d) R+W of this rank's band of the step's pictures"},
        "kernel_ms": {"inter": float(kern[0]), "intra": float(kern[1]), "deblock": float(kern[2]),
                      "batch_wall": float(kern[3])},
        "exchange": {"mode": exchange if world > 1 else None, "halo_mb_rows": halo, "max_abs_mvy_qpel": mvy,
                     "impl": (impl if world > 1 else None), "impl_note": impl_note,
                     "bytes_in_per_rank_per_step": xin,
                     "ops_per_step": xops},
        "cpu_baseline": cpu,
        "cpu_baseline_threads": cpu_mt,
        "verified_vs_oracle": verified,
    }


def xch_ops(xch, bands, rank, halo, exchange):
    """Transfers one group's exchange posts: the library's (h264r_group, point-to-point in both
    modes), or the torch implementation's (one all-gather, or one send / receive per peer)."""
    if xch.impl == "abi":
        return len(xch.need) + len(xch.give)
    return 1 if exchange == "allgather" else len(groups_peers(bands, rank, halo))


def groups_peers(bands, rank, halo):
    from h264r import dist as D
    need, give = D.halo_plan(bands, rank, halo)
    return sorted(set(need) | set(give))


def spawn_ranks(args) -> int:
    """`bench.py --gpus N` without a launcher (WORLD_SIZE unset): start N ranks through
    torch.distributed.run as a CHILD process (nothing here has touched the GPU), wait, and exit
    with its status; rank 0 prints the JSON line on the inherited stdout."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def throughput_run(args, rank: int, world: int, local: int, cs, rehearse: bool, ranks: dict):
    """Throughput mode (the one-GPU headline; at N > 1 replicas, or slice bands with --shard
    slices): B pictures per rank per step, one h264r_decode_batch each.  Returns the JSON
    line's dict on rank 0, None on the other ranks."""
    import torch
    import torch.distributed as dist
    import h264r
    from h264r import batch as B
    from h264r import synth
    from h264r import dist as D

    L = h264r.lib()
    W, H = CONFIG_SIZE[args.config]
    # pictures per GPU per step: the order-dependent walks (deblocking wavefront, intra
    # levels) need many pictures in flight; 1080p config 2/3 batches of 1024 pictures
    # (~8 GB of HBM) beat 256 by ~12 % (profiles/r01_batch_sweep.txt).  Slice mode
    # holds world x nb pictures per rank, so configs 4/5 stay smaller.
    nb = args.batch or {2: 1024, 3: 1024, 4: 256, 5: 64}[args.config]
    cfg = synth.default_cfg(L, args.config, W, H)
    nmb = W * H
    shard = args.shard or ("slices" if world > 1 and cfg.deblock_idc != 0 and cfg.num_slices > 1 else "replicas")
    if shard == "slices" and cfg.deblock_idc == 0:
        raise SystemExit("slice sharding needs disable_deblocking_filter_idc 1/2 (configs 4, 5)")

    # inputs.  replicas: this rank's own pictures.  slices (weak scaling): every rank
    # holds the same world * nb pictures and reconstructs its band of slices of each.
    if shard == "replicas":
        pics = [synth.picture(L, cfg, i) for i in D.picture_share(rank, world, nb)]
    else:
        pics = [synth.picture(L, cfg, i) for i in range(world * nb)]
    npics = len(pics)
    refs = synth.refpics(L, cfg)
    rd = wr = 0
    for p in pics:
        r, w = synth.algo_bytes(L, p)
        rd += r
        wr += w
    band = (0, H)
    if shard == "slices":
        srow = pics[0].mbs["slice"].reshape(H, W)[:, 0]
        first = [0] + [r for r in range(1, H) if srow[r] != srow[r - 1]]
        bands = D.slice_bands(first, H, world)
        band = bands[rank]
        frac = (band[1] - band[0]) / H
        rd, wr = int(rd * frac), int(wr * frac)          # this rank's share (rows are uniform)

    dec = h264r.Decoder(local, W, H)
    # DPB slots as torch tensors (+ H264R_PLANE_SLACK).  Slice mode keeps three copies
    # E[0..2] of reference slot 0: step t predicts from E[t % 3] while the exchange of
    # step t's picture 0 lands in E[(t + 2) % 3] on a communication stream, so the
    # all-gather of step t overlaps the decode of step t + 1
    slack = 64
    plane_rows = (16 * H, 8 * H, 8 * H)
    row_bytes = (16 * W, 8 * W, 8 * W)

    def slot_planes(src, cap=None):
        out = []
        for k, a in enumerate(src):
            n = cap[k] if cap else a.size
            t = torch.zeros(n + slack, dtype=torch.uint8, device="cuda")
            t[: a.size].copy_(torch.from_numpy(np.ascontiguousarray(a).reshape(-1)))
            out.append(t)
        return out
    if not refs:                                   # all-intra (config 2): no reference picture
        ring = [[]]
    elif shard == "slices":
        caps = [D.slot_capacity(plane_rows[k], row_bytes[k], bands, (16, 8, 8)[k]) for k in range(3)]
        ring = [slot_planes(refs[0], caps) for _ in range(3)]
    else:
        ring = [slot_planes(refs[0])]
    others = [slot_planes(r) for r in refs[1:]]
    tabs = []
    for e in ring:
        tab = np.zeros(3 * 32, np.int64)
        for s_, planes in enumerate(([e] if e else []) + others):
            for k in range(3):
                tab[3 * s_ + k] = planes[k].data_ptr()
        tabs.append(torch.from_numpy(tab).to("cuda"))
    # placement experiment (box-to-box spread): H264R_BENCH_PAD_MB allocates a pad
    # before the batch and the library's scratch, shifting where every buffer lands in HBM
    pad_mb = int(os.environ.get("H264R_BENCH_PAD_MB", "0"))
    pad = torch.empty(pad_mb << 20, dtype=torch.uint8, device="cuda") if pad_mb > 0 else None
    host = B.pack(pics, h264r.quant_flat())
    db = B.to_device(host, npics, tabs[0].data_ptr())
    # the batch is resident in HBM now: keep only what the checks below read (three
    # pictures and the per-kernel algorithmic bytes), so a rank holds ~4 MB per picture once
    kbytes_all = kernel_bytes(pics, nmb)
    check_idx = sorted({0, npics // 2, npics - 1}) if shard == "replicas" else [0]
    check_pics = {i: pics[i] for i in check_idx}
    del host, pics
    stream = cs.cuda_stream
    comm = torch.cuda.Stream(device=local) if shard == "slices" else None
    stage = ([torch.zeros(max(b1 - b0 for b0, b1 in bands) * m * rb, dtype=torch.uint8, device="cuda")
              for m, rb in zip((16, 8, 8), row_bytes)] for _ in range(2)) if shard == "slices" else ()
    stage = list(stage)
    ev_dec, ev_ex = [], []
    nstep = [0]
    turn = GpuTurn(rehearse and world > 1)

    def step():
        t = nstep[0]
        nstep[0] += 1
        if shard == "slices" and t >= 2:
            cs.wait_event(ev_ex[t - 2])                # E[t % 3] and stage[t % 2] are free again
        db.batch.ref_planes = tabs[t % len(tabs)].data_ptr()
        if band[1] > band[0]:
            with turn:
                dec.decode_batch(db.batch, stream, rows=None if band == (0, H) else band)
        if shard != "slices":
            return
        # exchange: this rank's band of picture 0 staged (one small D2D copy, so the next
        # step may overwrite the output planes), then one RCCL all-gather per plane into
        # E[(t + 2) % 3] on the communication stream
        outs = (db.tensors["out_y"][0], db.tensors["out_u"][0], db.tensors["out_v"][0])
        st = stage[t % 2]
        for k, m in enumerate((16, 8, 8)):
            a0, a1 = band[0] * m * row_bytes[k], band[1] * m * row_bytes[k]
            st[k][: a1 - a0].copy_(outs[k][a0:a1])
        ev = torch.cuda.Event()
        ev.record(cs)
        ev_dec.append(ev)
        comm.wait_event(ev)
        with torch.cuda.stream(comm):
            for k, m in enumerate((16, 8, 8)):
                D.allgather_into_slot(st[k], ring[(t + 2) % 3][k], bands, rank, m, row_bytes[k])
            ex = torch.cuda.Event()
            ex.record(comm)
        ev_ex.append(ex)

    # correctness first (refs as generated).  Replicas: pictures 0, middle and last of the
    # batch vs the oracle (the largest offsets are checked too).  Slices: after
    # the exchange, the picture every rank received in E[2] vs the oracle's picture 0.
    verified = None
    if not args.no_verify:
        step()
        torch.cuda.synchronize()
        dec.check()
        if rank == 0:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import _oracle as O
            verified = True
            for i, p in check_pics.items():
                want = O.decode(p, refs)
                if shard == "slices":
                    got = [ring[2][k][: plane_rows[k] * row_bytes[k]].cpu().numpy().reshape(want[k].shape)
                           for k in range(3)]
                else:
                    got = db.planes(i)
                verified &= all(np.array_equal(got[k], want[k]) for k in range(3))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # timed region: barrier + sync on both sides, exactly `steps` steps.  Every kernel
    # launch inside it is bracketed by HIP events on the stream it runs on; the
    # library averages those per step (per-kernel busy time + whole-batch wall time).
    dec.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    # a bounded device-side wait that expired would have cut a launch short (fast and
    # wrong): the timed steps only count if none did
    dec.check()
    kern = np.array(dec.last_timing()) if band[1] > band[0] else np.zeros(4)
    dec.set_timing(False)
    dt = D.max_over_ranks(dt, device="cpu" if rehearse else "cuda")

    total_mbs = (world * nb if shard == "replicas" else npics) * nmb * args.steps
    value = total_mbs / dt
    ms_per_step = dt / args.steps * 1e3
    step_bytes = rd + wr
    mbs_rank = (nb * nmb) if shard == "replicas" else int(npics * nmb * (band[1] - band[0]) / H)
    # roofline: the path is one launch sequence per step; its algorithmic
    # bytes = sum over the batch's MBs of R + W (8(d) formula, exact over the synthetic
    # batch), divided by the sequence's device time (HIP events around the whole launch
    # sequence on its stream, averaged over the timed steps)
    achieved = step_bytes / (kern[3] * 1e-3) / 1e9 if kern[3] > 0 else 0.0
    # per-kernel split of the same 8(d) bytes (kernel_bytes: R to the reconstructing kernel,
    # W to deblocking; the parts add up to the path's bytes), over each kernel's own event time
    kbytes = [int(k * (band[1] - band[0]) / H) for k in kbytes_all]
    # the library deblocks launches of fewer than H264R_DB2S_MAX (default 512) x 68 picture-MB-rows
    # with the split walk (k_deblock2y + k_deblock2c), larger ones with k_deblock2 (h264r_host.hip)
    prow = npics * (band[1] - band[0])
    dbk_k = (["k_deblock2y", "k_deblock2c"] if prow < int(os.environ.get("H264R_DB2S_MAX", "512")) * 68
             else ["k_deblock2"] if prow >= int(os.environ.get("H264R_DEBLOCK2_MIN", "8")) * 68 else ["k_deblock"])
    dbk = " + ".join(dbk_k)
    inter_k = ["k_inter4r"]
    names = [" + ".join(inter_k), "intra (k_level + k_intra_levels + k_intra_pic)", dbk]
    kern_names = [inter_k + ["k_inter_sp"], ["k_level", "k_level_scatter", "k_intra_levels", "k_intra_pic"],
                  dbk_k]
    # HBM traffic per launch sequence from the PMC counters of the committed profile run
    # (tools/pmc.sh + tools/pmc_summary.py --json): per-MB FETCH_SIZE (doubled, gfx950) +
    # WRITE_SIZE of every kernel of the sequence, times the MBs this rank processed
    traffic, traffic_src, ktraffic = None, None, [None, None, None]
    kvalu = [None, None, None]
    tpath = args.traffic_json or os.path.join(ROOT, "profiles", "traffic.json")
    if not args.traffic_json and args.config != 3 and os.path.exists(os.path.join(ROOT, "profiles", f"traffic_c{args.config}.json")):
        tpath = os.path.join(ROOT, "profiles", f"traffic_c{args.config}.json")
    if os.path.exists(tpath):
        tj = json.load(open(tpath))
        if tj.get("survey_config", 3) == args.config:
            per = {k: v["traffic_bytes_per_mb"] for k, v in tj["kernels"].items()}
            traffic = int(sum(per.values()) * mbs_rank)
            ktraffic = [int(sum(per.get(n, 0) for n in kn) * mbs_rank) for kn in kern_names]
            traffic_src = f"{os.path.basename(tpath)} ({tj.get('source')}): all kernels of the sequence"
            vper = {k: v.get("valu_per_mb") for k, v in tj["kernels"].items()}
            if all(vper.get(n) is not None for kn in kern_names for n in kn if n in vper):
                kvalu = [sum(vper.get(n) or 0.0 for n in kn) for kn in kern_names]
    kernels = {}
    for i, nme in enumerate(names):
        ach = kbytes[i] / (kern[i] * 1e-3) / 1e9 if kern[i] > 0 else 0.0
        kernels[nme] = {"ms": float(kern[i]), "algo_bytes": kbytes[i], "achieved": ach,
                        "frac": ach / HBM_PEAK_GBS, "traffic": ktraffic[i]}
        # the second roof: VALU issue.  A wave64 VALU instruction occupies
        # its SIMD-32 for 2 cycles (MI355X_MICROARCH.md, wave scheduling), so the chip issues at
        # most 256 CUs x 4 SIMDs x 2.4 GHz / 2 wave-instructions per second; valu_floor_ms is
        # the kernel's PMC VALU count (profiles/traffic.json) at that rate
        if kvalu[i] is not None and kern[i] > 0:
            floor_ms = kvalu[i] * mbs_rank / VALU_ISSUE_PER_S * 1e3
            kernels[nme].update({"valu_per_mb": kvalu[i], "valu_floor_ms": floor_ms,
                                 "valu_frac": floor_ms / float(kern[i])})

    # a measured copy-kernel peak beside the spec peak (device-to-device copy
    # of 1 GiB, read + write bytes over its HIP-event time, best of 5), outside the timed region
    copy_peak = None
    if band[1] > band[0]:
        src = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
        dst = torch.empty_like(src)
        best = None
        for _ in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            dst.copy_(src)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        copy_peak = 2 * src.numel() / (best * 1e-3) / 1e9
        del src, dst

    cpu = cpu_mt = None
    if rank == 0 and world == 1 and not args.no_cpu:
        done, el, ncpu = cpu_baseline(cfg, refs, args.cpu_seconds)
        cpu = {"value": done / el, "unit": "macroblocks/s", "cores": 1, "kind": "port",
               "sample": f"{ncpu} pictures of the same {CONFIG_NAMES[args.config]} workload "
                         f"({ncpu * nmb} MBs, {el:.1f} s) decoded by oracle/h264r_oracle.c (1 thread) "
                         f"on {cpu_model()}"}
        # the box gives one GPU's job a 16-CPU share (os.cpu_count() shows the whole machine)
        thr = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        done, el, ncpu = cpu_baseline_threads(cfg, refs, args.cpu_seconds / 2, thr)
        cpu_mt = {"value": done / el, "unit": "macroblocks/s", "cores": thr, "kind": "port",
                  "sample": f"{ncpu} pictures ({ncpu * nmb} MBs, {el:.1f} s) over {thr} threads, "
                            f"oracle_decode_pictures, on {cpu_model()}"}

    latency = None
    if rank == 0 and world == 1 and args.latency_pictures > 0 and shard == "replicas":
        ms, nl, lver = latency_chain(dec, L, cfg, refs, stream, args.latency_pictures,
                                     0 if args.no_verify else 3)
        latency = {"ms_per_picture": ms, "pictures": nl, "macroblocks_per_s": nmb / (ms * 1e-3),
                   "verified_vs_oracle": lver,
                   "workload": f"dependent chain of {CONFIG_NAMES[args.config]}, one picture per launch "
                               "(slot 0 = previous decoded picture)"}

    if rank == 0:
        out = {
            "metric": "macroblocks/s (decode reconstruct, post-entropy) 1080p P-frame; % HBM roofline",
            "value": value, "unit": "macroblocks/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded SURVEY 8(d) generator, arrow-h264_amd/csrc/synth.c)",
            "config": {"workload": CONFIG_NAMES[args.config], "survey_config": args.config,
                       "width_mbs": W, "height_mbs": H, "pictures_per_gpu": nb,
                       "parallelism": (f"{shard}{world}" if world > 1 else "single"),
                       "pictures_per_step": world * nb if shard == "replicas" else npics,
                       "rows_this_rank": list(band)},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": f"h264r_decode_batch launch sequence ({', '.join(inter_k)}, k_inter_sp, "
                                   f"k_level, k_intra_levels, k_intra_pic, {dbk})",
                         "kernel_ms": float(kern[3]), "kernel_algo_bytes": int(step_bytes),
                         "bytes_per_mb": step_bytes / max(mbs_rank, 1),
                         "numerator": "SURVEY 8(d) R+W summed exactly over the batch's MBs",
                         "path_frac_wall": value / world * step_bytes / max(mbs_rank, 1) / (HBM_PEAK_GBS * 1e9),
                         "read_frac": (rd / (kern[3] * 1e-3) / 1e9 / HBM_PEAK_GBS) if kern[3] > 0 else 0.0,
                         "valu_floor_ms": (sum(k["valu_floor_ms"] for k in kernels.values())
                                           if all("valu_floor_ms" in k for k in kernels.values()) else None),
                         "copy_peak_measured": copy_peak,
                         "frac_of_copy_peak": (achieved / copy_peak) if copy_peak else None,
                         "kernels": kernels},
            "kernel_ms": {"inter": float(kern[0]), "intra": float(kern[1]), "deblock": float(kern[2]),
                          "batch_wall": float(kern[3])},
            "cpu_baseline": cpu,
            "cpu_baseline_threads": cpu_mt,
            "latency": latency,
            "verified_vs_oracle": verified,
            "distributed": ranks,
        }
        vf = out["roofline"]["valu_floor_ms"]
        if vf:
            # the HBM fraction the path could reach if every kernel issued VALU back to back at
            # today's instruction counts (the ceiling the second roof puts on the first)
            out["roofline"]["frac_ceiling_at_valu_floor"] = step_bytes / (vf * 1e-3) / 1e9 / HBM_PEAK_GBS
        return out
    return None

def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs = ranks; without WORLD_SIZE in the environment bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=None, choices=[2, 3, 4, 5],
                    help="SURVEY 8(d) workload (default: 3 at one GPU, 5 at N > 1)")
    ap.add_argument("--mode", choices=["throughput", "chain"], default=None,
                    help="throughput: independent pictures sharing a reference set (default at one GPU); "
                         "chain: dependent chains, slice-sharded over the ranks (default at N > 1)")
    ap.add_argument("--batch", type=int, default=0, help="throughput mode: pictures per GPU per step (default 1024 for configs 2/3, 256 for 4, 64 at 2160p)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16, help="threads of the multi-threaded CPU baseline")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--latency-pictures", type=int, default=32,
                    help="length of the dependent-chain latency run (rank 0, N=1; 0 = skip)")
    ap.add_argument("--traffic-json", default=None, help="PMC traffic summary (default profiles/traffic.json, "
                    "profiles/traffic_c<config>.json for other configs when present)")
    ap.add_argument("--chain", type=int, default=0,
                    help="chain mode with this many chains in all (a multiple of --chain-groups); "
                         "default chains-per-gpu x N")
    ap.add_argument("--chain-groups", type=int, default=1,
                    help="chain mode: launches per step (groups of chains); with 2 or more the exchange of one "
                         "group overlaps the decode of the next")
    ap.add_argument("--chains-per-gpu", type=int, default=32,
                    help="chain mode: chains per GPU (weak scaling: the job holds chains-per-gpu x N chains)")
    ap.add_argument("--exchange", choices=["halo", "allgather"], default="halo",
                    help="chain mode at N > 1: rows within the motion vectors' reach from the neighbouring "
                         "bands (point-to-point), or every band (all-gather)")
    ap.add_argument("--exchange-impl", choices=["abi", "torch"], default="abi",
                    help="chain mode at N > 1: the exchange in the library (include/h264r_group.h: RCCL "
                         "send / recv between pack and unpack kernels) or in torch.distributed calls")
    ap.add_argument("--no-n1", action="store_true", help="chain mode at N > 1: skip the one-GPU line of the same mode")
    ap.add_argument("--no-sliced", action="store_true",
                    help="N > 1 default: skip the slice-sharded config-5 chain line reported beside the replicas")
    ap.add_argument("--shard", choices=["replicas", "slices"], default=None,
                    help="throughput mode at N>1: independent pictures per GPU, or slice bands of shared pictures "
                         "(default: slices for configs 4/5, replicas for 2/3)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    mode = "chain" if args.chain else (args.mode or "throughput")
    # N > 1 with no --mode: the headline workload as replicas (the value the scaling curve
    # compares with the one-GPU line), plus the slice-sharded dependent-chain run of config 5
    # beside it in the same JSON line (`slice_sharded`)
    sliced = world > 1 and args.mode is None and not args.chain and not args.no_sliced
    if args.config is None:
        args.config = 5 if mode == "chain" else 3

    import torch
    import torch.distributed as dist
    import h264r
    from h264r import batch as B
    from h264r import synth
    from h264r import dist as D

    # H264R_BENCH_REHEARSE=1 (testing the N > 1 code path on a one-GPU box): every rank on
    # device 0, gloo instead of RCCL (RCCL refuses two ranks on one GPU); never a measurement
    rehearse = os.environ.get("H264R_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    # every device operation of this process (allocations, uploads, decode, exchange,
    # checks) goes on ONE explicit stream, which is also the stream the library launches
    # on: torch's default stream is the legacy NULL stream, which the C ABI would map to
    # the context's own stream (unordered with torch's fills and copies)
    cs = torch.cuda.Stream(device=local)
    torch.cuda.set_stream(cs)
    backend = None
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        backend = dist.get_backend()
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
        dist.barrier()                                  # communicators up before any P2P
    ranks = {"backend": backend, "rccl_ranks": dist.get_world_size() if backend == "nccl" else 0,
             "ranks": world, "rehearsal": rehearse}

    if mode == "chain":
        nch = args.chain or args.chains_per_gpu * world
        out = chain_run(args, rank, world, local, cs, rehearse, nch, args.config, args.exchange)
        out["distributed"] = ranks
        if world > 1 and not args.no_n1:
            # the one-GPU line of the same mode and per-GPU load (weak scaling reference), on
            # rank 0 alone after the N-rank run; the other ranks wait at the barrier
            if rank == 0:
                n1 = chain_run(args, 0, 1, local, cs, rehearse, nch // world, args.config, args.exchange)
                out["same_mode_n1"] = {k: n1[k] for k in ("value", "ms_per_step", "verified_vs_oracle", "kernel_ms")}
                out["same_mode_n1"]["chains"] = n1["config"]["chains"]
                out["scaling_vs_same_mode_n1"] = out["value"] / (world * n1["value"])
            dist.barrier()
        if rank == 0:
            print(json.dumps(out))
        if world > 1:
            dist.destroy_process_group()
        return 0

    out = throughput_run(args, rank, world, local, cs, rehearse, ranks)
    if sliced:
        # the slice-sharded line: config 5 chains, each rank its band of every picture, the halo
        # rows over RCCL; then rank 0 alone runs the same mode at one GPU (its weak-scaling
        # reference).  Reported beside the headline, which stays the replicas of config 3.
        torch.cuda.empty_cache()
        dist.barrier()
        nch = args.chains_per_gpu * world
        sl = chain_run(args, rank, world, local, cs, rehearse, nch, 5, args.exchange)
        if rank == 0:
            n1 = chain_run(args, 0, 1, local, cs, rehearse, nch // world, 5, args.exchange)
            keep = ("metric", "value", "unit", "ms_per_step", "config", "roofline", "kernel_ms", "exchange",
                    "verified_vs_oracle")
            out["slice_sharded"] = {k: sl[k] for k in keep}
            out["slice_sharded"]["same_mode_n1"] = {k: n1[k] for k in ("value", "ms_per_step", "verified_vs_oracle",
                                                                      "kernel_ms", "cpu_baseline")}
            out["slice_sharded"]["same_mode_n1"]["chains"] = n1["config"]["chains"]
            out["slice_sharded"]["scaling_vs_same_mode_n1"] = sl["value"] / (world * n1["value"])
        dist.barrier()
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
