#!/usr/bin/env python3
"""Benchmark: macroblocks/s of post-entropy reconstruction (MC + IDCT + intra +
deblock) on MI355X, BASELINE.json's metric.

A step = one h264r_decode_batch over a batch of synthetic pictures already
resident in HBM (SURVEY 8(d) throughput mode: B independent pictures sharing a
reference set).  Default workload: SURVEY config 3, 1080p (120x68 MBs) IPPP
Main P pictures, B = 1024 per GPU (about 8 GB of HBM: the order-dependent walks
need many pictures in flight to fill 256 CUs).

Multi-GPU (torchrun, one process per GPU): config 3 uses deblocking across the
whole picture (disable_deblocking_filter_idc 0), which chains every MB of a
picture (deblock.cc:547-551), so N > 1 runs N independent replicas (one stream
per GPU, weak scaling, no data-path collective); see DESIGN.md.

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


def chain_bench(args, rank: int, world: int, local: int, cs, rehearse: bool) -> dict:
    """--chain K: K dependent chains per step, slice-sharded over the ranks (DESIGN
    section 6).  Chain k's picture t predicts from its picture t-1 (DPB slot k): a rank decodes
    its slice band of the K pictures, then ONE all-gather per plane brings every rank's band
    of all K pictures into every rank's chain slots before any chain's next picture may
    start -- one exchange per reference picture, on the dependency path.  The chains are
    split into two groups whose batches alternate on the decode stream, so the exchange of
    one group (communication stream) overlaps the decode of the other.  Each group keeps
    two slot sets (ping-pong: step t reads set t % 2, its exchange fills set (t+1) % 2)."""
    import torch
    import h264r
    from h264r import batch as B
    from h264r import synth
    from h264r import dist as D
    L = h264r.lib()
    W, H = CONFIG_SIZE[args.config]
    cfg = synth.default_cfg(L, args.config, W, H)
    refs = synth.refpics(L, cfg)
    if not refs:
        raise SystemExit("--chain needs inter pictures (configs 3, 4, 5)")
    kg = args.chain // 2
    nmb = W * H
    base = [synth.picture(L, cfg, i) for i in range(2 * kg)]
    srow = base[0].mbs["slice"].reshape(H, W)[:, 0]
    first = [0] + [r for r in range(1, H) if srow[r] != srow[r - 1]]
    bands = D.slice_bands(first, H, world) if world > 1 else [(0, H)]
    band = bands[rank]
    if world > 1 and cfg.deblock_idc == 0:
        raise SystemExit("slice sharding needs disable_deblocking_filter_idc 1/2 (configs 4, 5)")
    slack = 64
    pbytes = (256 * nmb, 64 * nmb, 64 * nmb)
    rows_per_mb, row_bytes = (16, 8, 8), (16 * W, 8 * W, 8 * W)
    dec = h264r.Decoder(local, W, H)
    static = []
    for r in refs[1:]:
        static.append([torch.from_numpy(np.concatenate([a.reshape(-1), np.zeros(slack, np.uint8)])).to("cuda")
                       for a in r])
    groups = []
    for g in range(2):
        pics = []
        for k in range(kg):
            p = base[g * kg + k]
            p.slices = D.chain_slots(p.slices, k, kg)
            pics.append(p)
        # two slot sets per plane: [kg][plane + slack], every chain starting from refs[0]
        sets = []
        for _ in range(2):
            planes = []
            for k3 in range(3):
                t = torch.zeros((kg, pbytes[k3] + slack), dtype=torch.uint8, device="cuda")
                t[:, :pbytes[k3]].copy_(torch.from_numpy(refs[0][k3].reshape(1, -1)).expand(kg, -1))
                planes.append(t)
            sets.append(planes)
        tabs = []
        for si in range(2):
            tab = np.zeros(3 * 32, np.int64)
            for k in range(kg):
                for k3 in range(3):
                    tab[3 * k + k3] = sets[si][k3][k].data_ptr()
            for j, planes in enumerate(static):
                for k3 in range(3):
                    tab[3 * (kg + j) + k3] = planes[k3].data_ptr()
            tabs.append(torch.from_numpy(tab).to("cuda"))
        db = B.to_device(B.pack(pics, h264r.quant_flat()), kg, tabs[0].data_ptr())
        groups.append(dict(pics=pics, sets=sets, tabs=tabs, db=db, ev_ex=[]))
    comm = torch.cuda.Stream(device=local)
    stream = cs.cuda_stream
    nstep = [0]

    def step():
        t = nstep[0]
        nstep[0] += 1
        for G in groups:
            if t >= 1:
                cs.wait_event(G["ev_ex"][t - 1])       # this chain group's previous pictures are in place
            G["db"].batch.ref_planes = G["tabs"][t % 2].data_ptr()
            if band[1] > band[0]:
                dec.decode_batch(G["db"].batch, stream, rows=None if band == (0, H) else band)
            ev = torch.cuda.Event()
            ev.record(cs)
            comm.wait_event(ev)
            with torch.cuda.stream(comm):
                outs = (G["db"].tensors["out_y"], G["db"].tensors["out_u"], G["db"].tensors["out_v"])
                for k3 in range(3):
                    D.chain_exchange(outs[k3], G["sets"][(t + 1) % 2][k3], bands, rank, pbytes[k3],
                                     pbytes[k3] + slack, rows_per_mb[k3], row_bytes[k3])
                ex = torch.cuda.Event()
                ex.record(comm)
            G["ev_ex"].append(ex)

    verified = None
    if not args.no_verify:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import _oracle as O
        verified = True
        G = groups[0]
        prev = refs[0]
        for t in range(2):                             # chain 0 of group 0, two dependent pictures
            step()
            torch.cuda.synchronize()
            dec.check()
            if rank == 0:
                slot_refs = [prev] + [refs[0]] * (kg - 1) + list(refs[1:])
                want = O.decode(G["pics"][0], slot_refs)
                got = [G["sets"][(t + 1) % 2][k3][0, :pbytes[k3]].cpu().numpy() for k3 in range(3)]
                verified &= all(np.array_equal(got[k3], want[k3].reshape(-1)) for k3 in range(3))
                prev = want
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
    kern = np.array(dec.last_timing()) * 2 if band[1] > band[0] else np.zeros(4)   # two launches per step
    dec.set_timing(False)
    dt = D.max_over_ranks(dt, device="cpu" if rehearse else "cuda")
    rd = wr = 0
    for p in base:
        r, w = synth.algo_bytes(L, p)
        rd, wr = rd + r, wr + w
    total_mbs = 2 * kg * nmb * args.steps
    value = total_mbs / dt
    frac_rows = (band[1] - band[0]) / H
    step_bytes = int((rd + wr) * frac_rows)
    achieved = step_bytes / (kern[3] * 1e-3) / 1e9 if kern[3] > 0 else 0.0
    return {
        "metric": "macroblocks/s (decode reconstruct, post-entropy) 1080p P-frame; % HBM roofline",
        "value": value, "unit": "macroblocks/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic (seeded SURVEY 8(d) generator, arrow-h264_amd/csrc/synth.c)",
        "config": {"workload": f"{CONFIG_NAMES[args.config]}, {2 * kg} dependent chains (each picture predicts "
                               "from its chain's previous decoded picture; one all-gather per plane per step)",
                   "survey_config": args.config, "width_mbs": W, "height_mbs": H, "mode": "chain",
                   "chains": 2 * kg, "parallelism": f"slices{world}" if world > 1 else "single",
                   "rows_this_rank": list(band), "bands": [list(b) for b in bands]},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": "h264r_decode_batch launch sequences of the two chain groups",
                     "kernel_ms": float(kern[3]), "kernel_algo_bytes": step_bytes,
                     "numerator": "SURVEY 8(d) R+W of this rank's band of the step's pictures"},
        "kernel_ms": {"inter": float(kern[0]), "intra": float(kern[1]), "deblock": float(kern[2]),
                      "batch_wall": float(kern[3])},
        "exchange_per_step": {"collectives": 3 if world > 1 else 0,
                              "bytes_per_rank": int(sum(pbytes) * 2 * kg * frac_rows)},
        "cpu_baseline": None,
        "verified_vs_oracle": verified,
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3, choices=[2, 3, 4, 5])
    ap.add_argument("--batch", type=int, default=0, help="pictures per GPU per step (default 1024 for configs 2/3, 256 for 4, 64 at 2160p)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16, help="threads of the multi-threaded CPU baseline")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--latency-pictures", type=int, default=32,
                    help="length of the dependent-chain latency run (rank 0, N=1; 0 = skip)")
    ap.add_argument("--traffic-json", default=None, help="PMC traffic summary (default profiles/traffic.json)")
    ap.add_argument("--chain", type=int, default=0,
                    help="dependent-chain mode: this many chains (even, <= 60) advance one picture per step, "
                         "slice-sharded with one all-gather per reference picture (see chain_bench)")
    ap.add_argument("--shard", choices=["replicas", "slices"], default=None,
                    help="N>1 placement: independent pictures per GPU, or slice bands of shared pictures "
                         "(default: slices for configs 4/5, replicas for 2/3)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

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
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    if args.chain:
        if args.chain % 2 or not 2 <= args.chain <= 60:
            raise SystemExit("--chain takes an even number of chains, 2..60")
        out = chain_bench(args, rank, world, local, cs, rehearse)
        if rank == 0:
            print(json.dumps(out))
        if world > 1:
            dist.destroy_process_group()
        return 0

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

    def step():
        t = nstep[0]
        nstep[0] += 1
        if shard == "slices" and t >= 2:
            cs.wait_event(ev_ex[t - 2])                # E[t % 3] and stage[t % 2] are free again
        db.batch.ref_planes = tabs[t % len(tabs)].data_ptr()
        if band[1] > band[0]:
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
    # the library deblocks batches of >= H264R_DEBLOCK2_MIN pictures (default 192) with
    # k_deblock2, smaller ones with k_deblock (include/h264r.h)
    # (k_deblock3 under H264R_DEBLOCK3=1); the deblocking records come from k_dbinfo before
    # k_inter4r (H264R_DBINFO=1, the default) or from k_inter4 itself (0)
    row_walk = "k_deblock3" if os.environ.get("H264R_DEBLOCK3", "0") not in ("", "0") else "k_deblock2"
    dbk = row_walk if npics >= int(os.environ.get("H264R_DEBLOCK2_MIN", "192")) else "k_deblock"
    inter_k = ["k_inter4"] if os.environ.get("H264R_DBINFO", "1") == "0" else ["k_dbinfo", "k_inter4r"]
    names = [" + ".join(inter_k), "intra (k_level + k_intra_levels + k_intra_pic)", dbk]
    kern_names = [inter_k + ["k_inter_sp"], ["k_level", "k_level_scan", "k_level_scatter", "k_intra_levels", "k_intra_pic"],
                  [dbk]]
    # HBM traffic per launch sequence from the PMC counters of the committed profile run
    # (tools/pmc.sh + tools/pmc_summary.py --json): per-MB FETCH_SIZE (doubled, gfx950) +
    # WRITE_SIZE of every kernel of the sequence, times the MBs this rank processed
    traffic, traffic_src, ktraffic = None, None, [None, None, None]
    tpath = args.traffic_json or os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tpath):
        tj = json.load(open(tpath))
        if tj.get("survey_config", 3) == args.config:
            per = {k: v["traffic_bytes_per_mb"] for k, v in tj["kernels"].items()}
            traffic = int(sum(per.values()) * mbs_rank)
            ktraffic = [int(sum(per.get(n, 0) for n in kn) * mbs_rank) for kn in kern_names]
            traffic_src = f"{os.path.basename(tpath)} ({tj.get('source')}): all kernels of the sequence"
    kernels = {}
    for i, nme in enumerate(names):
        ach = kbytes[i] / (kern[i] * 1e-3) / 1e9 if kern[i] > 0 else 0.0
        kernels[nme] = {"ms": float(kern[i]), "algo_bytes": kbytes[i], "achieved": ach,
                        "frac": ach / HBM_PEAK_GBS, "traffic": ktraffic[i]}

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
                         "copy_peak_measured": copy_peak,
                         "frac_of_copy_peak": (achieved / copy_peak) if copy_peak else None,
                         "kernels": kernels},
            "kernel_ms": {"inter": float(kern[0]), "intra": float(kern[1]), "deblock": float(kern[2]),
                          "batch_wall": float(kern[3])},
            "cpu_baseline": cpu,
            "cpu_baseline_threads": cpu_mt,
            "latency": latency,
            "verified_vs_oracle": verified,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
