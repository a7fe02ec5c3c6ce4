"""GPU path (lib/libh264r.so on gfx950) against the reference fixtures and the oracle.

Bit-exact on every sample: this is integer work.  Full BASELINE sizes (1080p,
2160p) are checked sample-for-sample against the oracle, which finishes them in
seconds.
"""
import hashlib
import itertools
import json
import os

import numpy as np
import pytest

import _oracle as O
import h264r
from h264r import _abi as A
from h264r import batch as B
from h264r import synth

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))["fixtures"]


def md5(a):
    return hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def L():
    h264r.build()
    return h264r.lib()


@pytest.fixture(scope="module")
def dec(L):
    d = h264r.Decoder(0, 240, 135)
    yield d
    d.close()


@pytest.fixture(scope="module")
def dec444(L):
    """A 4:4:4 context (chroma_format_idc 3): each colour plane decoded as luma."""
    d = h264r.Decoder(0, 240, 135, chroma_format=3)
    yield d
    d.close()


@pytest.fixture(scope="module")
def dec400(L):
    """A 4:0:0 context (chroma_format_idc 0): the luma pass alone."""
    d = h264r.Decoder(0, 240, 135, chroma_format=0)
    yield d
    d.close()


@pytest.fixture(scope="module")
def dec422(L):
    """A 4:2:2 context (chroma_format_idc 2): the luma pass, then k_c422_inter / k_c422_intra / k_c422_db."""
    d = h264r.Decoder(0, 240, 135, chroma_format=2)
    yield d
    d.close()


def first_diff(a, b, n, nh=None):
    bad = np.argwhere(a != b)
    if not len(bad):
        return None
    y, x = bad[0]
    return (f"{len(bad)} samples differ, first at (x={x}, y={y}) MB ({x // n}, {y // (nh or n)}): "
            f"gpu={a[y, x]} want={b[y, x]}")


@pytest.mark.parametrize("fx", GOLDEN, ids=[f"{f['name']}[{f['index']}]" for f in GOLDEN])
def test_gpu_matches_reference_fixture(L, dec, dec444, dec422, dec400, fx):
    cfg = A.SynthCfg.from_dict(fx["cfg"])
    dec = {0: dec400, 2: dec422, 3: dec444}.get(A.idc_of(cfg.chroma_format), dec)
    p = synth.picture(L, cfg, fx["index"])
    assert synth.input_digest(p) == fx["input_md5"]
    refs = synth.refpics(L, cfg)
    qm = fx.get("qmatrix")
    quant = h264r.quant_lists(qm["m4"], qm["m8"]) if qm else h264r.quant_flat()
    oquant = O.quant_lists(qm["m4"], qm["m8"]) if qm else None
    dec.assign_quant_params(quant)
    try:
        out = dec.decode_picture(p, refs)
        got = {k: md5(out[i]) for i, k in enumerate("YUV")}
        rec = dec.decode_picture(p, refs, no_deblock=True) if got != fx["out_md5"] else None
    finally:
        dec.assign_quant_params(h264r.quant_flat())
    if got != fx["out_md5"]:
        ref_rec = O.decode(p, refs, stage="recon", quant=oquant)
        ref_out = O.decode(p, refs, quant=oquant)
        msgs = []
        for i, k in enumerate("YUV"):
            n, nh = (16, 16) if i == 0 else A.chroma_mb(A.idc_of(cfg.chroma_format))
            d = first_diff(rec[i], ref_rec[i], n, nh)
            if d:
                msgs.append(f"recon {k}: {d}")
            d = first_diff(out[i], ref_out[i], n, nh)
            if d:
                msgs.append(f"final {k}: {d}")
        pytest.fail("; ".join(msgs) or "md5 mismatch")


# the deblocking schedules (include/h264r.h): one MB per 32 lanes, the band walk (8 lanes per MB row),
# the split walk (the luma and the chroma planes' walks as separate waves)
DEBLOCKS = (A.DBG_DEBLOCK_MB, A.DBG_DEBLOCK_ROWS, A.DBG_DEBLOCK_MB | A.DBG_DEBLOCK_GLOBAL, A.DBG_DEBLOCK_SPLIT)


def _batch_vs_oracle(L, dec, cidx, W, H, n, debug=0, deblocks=DEBLOCKS, qm=None, **over):
    """Decode n synthetic pictures in one batch under each deblocking schedule and compare
    every plane with the oracle's decode (qm: seed of explicit scaling lists)."""
    cfg = synth.default_cfg(L, cidx, W, H, **over)
    pics = [synth.picture(L, cfg, i) for i in range(n)]
    refs = synth.refpics(L, cfg)
    for s, (y, u, v) in enumerate(refs):
        dec.set_ref(s, y, u, v)
    lists = O.qmatrix(qm) if qm is not None else None
    host = B.pack(pics, h264r.quant_lists(*lists) if lists else h264r.quant_flat())
    want = [O.decode(p, refs, quant=O.quant_lists(*lists) if lists else None) for p in pics]
    for db_flag in deblocks:
        db = B.to_device(host, n, None)
        dec.set_debug(debug | db_flag)
        try:
            dec.decode_batch(db.batch)
            dec.check()
        finally:
            dec.set_debug(0)
        for i in range(n):
            got = db.planes(i)
            for k in range(3):
                d = first_diff(got[k], want[i][k], 16 if k == 0 else 8)
                assert d is None, f"deblock flag {db_flag} picture {i} plane {k}: {d}"


def _large_batch_vs_oracle(L, dec, cidx, W, H, n, nbase=8, debug=A.DBG_DEBLOCK_ROWS, rows=None, **over):
    """n pictures = nbase distinct ones repeated: every output is compared with the oracle's
    decode of its base picture (a large batch at little oracle cost).  rows: only that MB-row
    band is decoded (h264r_decode_batch_rows) and compared."""
    cfg = synth.default_cfg(L, cidx, W, H, **over)
    base = [synth.picture(L, cfg, i) for i in range(nbase)]
    refs = synth.refpics(L, cfg)
    for s, (y, u, v) in enumerate(refs):
        dec.set_ref(s, y, u, v)
    want = [O.decode(p, refs) for p in base]
    host = B.pack([base[i % nbase] for i in range(n)], h264r.quant_flat())
    db = B.to_device(host, n, None)
    dec.set_debug(debug)
    try:
        dec.decode_batch(db.batch, rows=rows)
        dec.check()
    finally:
        dec.set_debug(0)
    r0, r1 = rows if rows else (0, H)
    for i in range(n):
        got = db.planes(i)
        for k in range(3):
            m = 16 if k == 0 else 8
            d = first_diff(got[k][r0 * m:r1 * m], want[i % nbase][k][r0 * m:r1 * m], m)
            assert d is None, f"picture {i} plane {k}: {d}"


@pytest.mark.parametrize("cidx", [2, 3])
def test_gpu_large_batch_wide_rows(L, dec, cidx):
    """1080p-wide rows (W = 120 > 64) in a 256-picture batch of 32-row pictures: k_deblock2's
    XCD-local mode (64 groups of 4 pictures x 8 bands of 4 rows = 512 waves, 64 per XCD) and,
    all-intra, the walk's
    coarse band hand-off publishing mid-row (gstep 64 < W); every picture checked."""
    _large_batch_vs_oracle(L, dec, cidx, 120, 32, 256)


@pytest.mark.parametrize("cidx", [2, 3])
def test_gpu_large_batch_xcd_groups(L, dec, cidx):
    """464 CIF pictures (116 groups of 4 pictures x 5 bands of 4 MB rows, the last band 2 rows
    = 580 k_deblock2 waves): k_deblock2 in its XCD-local mode (groups on XCD g % 8,
    plain-store records) and the walk's coarse
    band hand-off (batches >= 128 pictures); every picture checked."""
    _large_batch_vs_oracle(L, dec, cidx, 22, 18, 464)


@pytest.mark.parametrize("cidx,n,debug", [
    (3, 1003, A.DBG_DEBLOCK_ROWS),
    (2, 1003, A.DBG_DEBLOCK_MB),
    (4, 1003, A.DBG_DEBLOCK_ROWS | A.DBG_DEBLOCK_GLOBAL),
    (3, 500, 0),
])
def test_gpu_overlapped_chunks(L, dec, cidx, n, debug):
    """The overlapped schedule (h264r_host.hip launch_all, H264R_DBG_OVERLAP): 1003 CIF pictures
    = 4 chunks of 251/251/251/250 (500 = 2 chunks), the side stream deblocking chunk k while the
    launch stream reconstructs chunk k + 1, under both deblocking schedules; every picture checked."""
    _large_batch_vs_oracle(L, dec, cidx, 22, 18, n, debug=debug | A.DBG_OVERLAP)


def test_gpu_overlapped_chunks_slice_band(L, dec):
    """The overlapped schedule over a slice band (h264r_decode_batch_rows, rows 5..14 of CIF
    pictures with 4 slices and idc 2 as bench.py's slice sharding has them)."""
    cfg = synth.default_cfg(L, 4, 22, 18, num_slices=4)
    srow = synth.picture(L, cfg, 0).mbs["slice"].reshape(18, 22)[:, 0]
    first = [r for r in range(1, 18) if srow[r] != srow[r - 1]]
    band = (first[0], first[2])
    _large_batch_vs_oracle(L, dec, 4, 22, 18, 1500, debug=A.DBG_DEBLOCK_ROWS | A.DBG_OVERLAP, rows=band, num_slices=4)


@pytest.mark.parametrize("n,nbase", [(6, 6), (1003, 8)])
def test_gpu_per_picture_dpb_tables(L, dec, n, nbase):
    """ABI 2 per-picture DPB tables (h264r_batch.ref_planes_stride = 3 x 32 pointers): picture i
    reads slot 0 from reference set i % 3 (three different pictures) and slot 1 from a shared
    one, so a kernel that ignored the stride, or a sub-batch of the overlapped schedule that
    did not advance the table pointer, would predict from the wrong planes.  1003
    pictures = four chunks of the overlapped schedule; every picture checked."""
    import torch
    W, H = 22, 18
    cfg = synth.default_cfg(L, 3, W, H)
    base = [synth.picture(L, cfg, i) for i in range(nbase)]
    refs = synth.refpics(L, cfg)
    rng = np.random.default_rng(7)
    alts = [refs[0]] + [tuple(rng.integers(0, 256, a.shape, dtype=np.uint8) for a in refs[0]) for _ in range(2)]
    slack = 64

    def dev(planes):
        return [torch.from_numpy(np.concatenate([a.reshape(-1), np.zeros(slack, np.uint8)])).to("cuda") for a in planes]
    alt_t = [dev(a) for a in alts]
    shared = dev(refs[1])
    tab = np.zeros((n, 3 * 32), np.int64)
    for i in range(n):
        for k in range(3):
            tab[i, k] = alt_t[i % 3][k].data_ptr()
            tab[i, 3 + k] = shared[k].data_ptr()
    tab_t = torch.from_numpy(tab.reshape(-1)).to("cuda")
    want = {}
    for i in range(min(n, 3 * nbase)):
        key = (i % nbase, i % 3)
        want[key] = O.decode(base[key[0]], [alts[key[1]], refs[1]])
    host = B.pack([base[i % nbase] for i in range(n)], h264r.quant_flat())
    for db_flag in (A.DBG_DEBLOCK_MB, A.DBG_DEBLOCK_ROWS | A.DBG_OVERLAP):
        db = B.to_device(host, n, tab_t.data_ptr())
        db.batch.ref_planes_stride = 3 * 32
        dec.set_debug(db_flag)
        try:
            dec.decode_batch(db.batch)
            dec.check()
        finally:
            dec.set_debug(0)
        for i in range(n):
            got = db.planes(i)
            w = want[(i % nbase, i % 3)]
            for k in range(3):
                d = first_diff(got[k], w[k], 16 if k == 0 else 8)
                assert d is None, f"deblock flag {db_flag} picture {i} (ref set {i % 3}) plane {k}: {d}"


def test_gpu_stray_env_selectors_are_inert(L, dec, monkeypatch):
    """The round-3 selectors that chose kernel variants (H264R_DBINFO, H264R_DEBLOCK3, H264R_PIPES)
    are gone from the library: set to values that once launched no deblocking records, they
    change nothing (a stale DbInfo must never be filtered with)."""
    for k, v in (("H264R_DBINFO", "3"), ("H264R_DEBLOCK3", "on"), ("H264R_PIPES", "4")):
        monkeypatch.setenv(k, v)
    _batch_vs_oracle(L, dec, 3, 22, 18, 3)
    _batch_vs_oracle(L, dec, 4, 22, 18, 2)


def test_gpu_batch_cif_p(L, dec):
    _batch_vs_oracle(L, dec, 3, 22, 18, 6)


def test_gpu_batch_cif_b_explicit_cip(L, dec):
    _batch_vs_oracle(L, dec, 4, 22, 18, 4, wp_mode=1, constrained_intra=1, num_refs=3, pcm_permille=20)


def test_gpu_batch_1080p_p(L, dec):
    """BASELINE config 3 size (1920x1088, IPPP Main distributions)."""
    _batch_vs_oracle(L, dec, 3, 120, 68, 3)


def test_gpu_batch_1080p_intra(L, dec):
    """BASELINE config 2 size (all-intra, 4x4 + 8x8)."""
    _batch_vs_oracle(L, dec, 2, 120, 68, 2)


def test_gpu_batch_1080p_p_intra_walk(L, dec):
    """The wavefront walk alone (no dependency-level schedule) on config 3."""
    _batch_vs_oracle(L, dec, 3, 120, 68, 2, debug=A.DBG_INTRA_WALK)


def test_gpu_batch_dense_intra_levels(L, dec):
    """P pictures with 60 % intra MBs: chains far deeper than the level launches, so
    the level schedule and the walk both take part in one picture."""
    _batch_vs_oracle(L, dec, 3, 40, 30, 3, intra_permille=600, pcm_permille=30)


_LEVELS_CODE = """
import sys
sys.path[:0] = [{root!r}, {tests!r}]
import test_gpu_parity as T, h264r
L = h264r.lib()
d = h264r.Decoder(0, 240, 135)
try:
    T._batch_vs_oracle(L, d, 3, 40, 30, 3, deblocks=(0,), intra_permille=600, pcm_permille=30)
    T._batch_vs_oracle(L, d, 3, 120, 68, 4, deblocks=(0,), intra_permille=300)
finally:
    d.close()
print("levels ok")
"""


@pytest.mark.parametrize("levels", ["8", "16"])
def test_gpu_batch_many_level_barriers(L, levels):
    """Every level from lists (H264R_LEVELS 8 / 16): the dense-intra pictures cross
    k_intra_levels' sharded grid barrier (8 shard counters + a top counter, k_picture.hip) up to
    15 times in one launch; the deeper MBs still go to the walk.  The library reads its knobs once
    per process (h264r_host.hip knobs()), so the case runs in a process of its own, and its
    H264R_VERBOSE report shows the level count each launch took."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = _LEVELS_CODE.format(root=os.path.join(os.path.dirname(here), "arrow-h264_amd"), tests=here)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=110,
                       env=dict(os.environ, H264R_LEVELS=levels, H264R_VERBOSE="1"))
    assert r.returncode == 0 and "levels ok" in r.stdout, r.stdout[-1500:] + r.stderr[-3000:]
    took = {ln for ln in r.stderr.splitlines() if "intra levels from lists" in ln}
    assert took and all(ln.startswith(f"h264r: {levels} intra levels") for ln in took), took


@pytest.mark.parametrize("n", [33, 70])
def test_gpu_batch_picture_groups(L, dec, n):
    """Batches spanning several picture groups of k_deblock2 (the last one ragged; 9 MB rows =
    bands of 4, 4 and 1 row) under both schedules; flag 0 takes the default for these sizes (the
    split walk for both: below H264R_DB2S_MAX x 68 picture-rows)."""
    _batch_vs_oracle(L, dec, 3, 11, 9, n, deblocks=(0, A.DBG_DEBLOCK_MB, A.DBG_DEBLOCK_ROWS), pcm_permille=20)


@pytest.mark.parametrize("cidx,over", [
    (2, dict(qp_min=0, qp_max=20, lossless_permille=500, pcm_permille=20)),
    (3, dict(qp_min=0, qp_max=20, lossless_permille=500, intra_permille=400, transform8x8=1)),
    (4, dict(qp_min=0, qp_max=20, lossless_permille=500)),
])
def test_gpu_batch_lossless(L, dec, cidx, over):
    """TransformBypassModeFlag MBs (F12, transform.cc:736-822) in every MB kind, CIF batches,
    through the level schedule and (all-intra) the walk."""
    _batch_vs_oracle(L, dec, cidx, 22, 18, 3, **over)


def test_gpu_batch_lossless_walk(L, dec):
    _batch_vs_oracle(L, dec, 3, 22, 18, 2, debug=A.DBG_INTRA_WALK, qp_min=0, qp_max=10, lossless_permille=600,
                     intra_permille=500, transform8x8=1)


@pytest.mark.parametrize("W,H,n,over", [
    (22, 18, 3, dict(num_slices=2, intra_permille=200, pcm_permille=20)),
    (120, 68, 2, dict(qp_min=0, qp_max=51)),
])
def test_gpu_batch_sp(L, dec, W, H, n, over):
    """SP pictures (F13: k_inter_sp, inverse_transform_sp transform.cc:1267-1300), switching and
    not, mixed with intra / PCM MBs, at CIF and config-3 size."""
    _batch_vs_oracle(L, dec, 3, W, H, n, sp_slices=1, **over)


def test_gpu_batch_1080p_b_scaling(L, dec):
    """Config 4 size with explicit (non-flat) scaling matrices."""
    _batch_vs_oracle(L, dec, 4, 120, 68, 2, qm=21)


def test_gpu_2160p_b_8slices(L, dec):
    """BASELINE config 5 size (3840x2160, 8 slices, idc 2)."""
    _batch_vs_oracle(L, dec, 5, 240, 135, 1)


@pytest.mark.parametrize("W,H", [(1, 1), (1, 7), (9, 1), (2, 2)])
def test_gpu_degenerate_sizes(L, dec, W, H):
    for cidx in (2, 3, 4):
        cfg = synth.default_cfg(L, cidx, W, H, pcm_permille=50, num_slices=1)
        p = synth.picture(L, cfg, 1)
        refs = synth.refpics(L, cfg)
        want = O.decode(p, refs)
        for flag in DEBLOCKS:
            got = dec.decode_picture(p, refs, debug=flag)
            for k in range(3):
                assert np.array_equal(got[k], want[k]), (cidx, flag, k)


def test_gpu_streaming_errors(L, dec):
    cfg = synth.default_cfg(L, 3, 4, 3)
    p = synth.picture(L, cfg, 0)
    dec.init(4, 3, p.pic, p.slices)
    with pytest.raises(h264r.H264RError) as e:
        dec.deblock_filter()          # no MB submitted
    assert e.value.status == A.ESTATE
    with pytest.raises(h264r.H264RError) as e:
        dec.deblock_filter()          # not inside a picture any more
    assert e.value.status == A.ESTATE
    with pytest.raises(h264r.H264RError) as e:
        dec.decode(0, p.mbs[:1], p.levels[:0], p.mv[:, :1, :1].repeat(16).reshape(2, 16), np.zeros((2, 16), np.int8))
    assert e.value.status == A.ESTATE


def test_single_hip_runtime_in_process(L, dec):
    """torch tensors and libh264r must share one HIP runtime (see h264r.lib())."""
    maps = open("/proc/self/maps").read()
    hip = {line.split()[-1] for line in maps.splitlines() if "libamdhip64" in line}
    assert len(hip) == 1, hip
    assert any("libh264r.so" in line for line in maps.splitlines())


def _slice_first_rows(p):
    W, H = p.cfg.width_mbs, p.cfg.height_mbs
    s = p.mbs["slice"].reshape(H, W)[:, 0]
    return [0] + [r for r in range(1, H) if s[r] != s[r - 1]]


@pytest.mark.parametrize("cidx,W,H,world", [(4, 120, 68, 4), (4, 120, 68, 2), (5, 240, 135, 8), (5, 240, 135, 3)])
def test_gpu_slice_bands_match_whole_picture(L, dec, cidx, W, H, world):
    """Slice-sharded decode (multi-GPU mode): each rank's band, decoded on
    its own by h264r_decode_batch_rows, equals those rows of the oracle's whole-picture
    decode and leaves every other row untouched."""
    from h264r import dist as D
    import torch
    n = 2
    cfg = synth.default_cfg(L, cidx, W, H)
    pics = [synth.picture(L, cfg, i) for i in range(n)]
    refs = synth.refpics(L, cfg)
    for s, (y, u, v) in enumerate(refs):
        dec.set_ref(s, y, u, v)
    want = [O.decode(p, refs) for p in pics]
    bands = D.slice_bands(_slice_first_rows(pics[0]), H, world)
    host = B.pack(pics, h264r.quant_flat())
    for (r0, r1), flag in itertools.product(bands, DEBLOCKS):
        if r1 == r0:
            continue
        db = B.to_device(host, n, None)
        dec.set_debug(flag)
        try:
            dec.decode_batch(db.batch, rows=(r0, r1))
            dec.check()
        finally:
            dec.set_debug(0)
        torch.cuda.synchronize()
        for i in range(n):
            got = db.planes(i)
            for k in range(3):
                m = 16 if k == 0 else 8
                inside = slice(r0 * m, r1 * m)
                d = first_diff(got[k][inside], want[i][k][inside], m)
                assert d is None, f"band {r0}..{r1} flag {flag} picture {i} plane {k}: {d}"
                outside = np.ones(got[k].shape[0], bool)
                outside[inside] = False
                assert not got[k][outside].any(), f"band {r0}..{r1} wrote outside its rows"


def test_gpu_band_across_filtered_edge_is_reported(L, dec):
    """Config 3 deblocks across the whole picture (idc 0): a band starting inside it
    would need rows it does not have, and h264r_check says so."""
    cfg = synth.default_cfg(L, 3, 22, 18, num_slices=2)
    p = synth.picture(L, cfg, 0)
    refs = synth.refpics(L, cfg)
    for s, (y, u, v) in enumerate(refs):
        dec.set_ref(s, y, u, v)
    r0 = _slice_first_rows(p)[1]
    for flag in DEBLOCKS:
        db = B.to_device(B.pack([p], h264r.quant_flat()), 1, None)
        dec.set_debug(flag)
        try:
            dec.decode_batch(db.batch, rows=(r0, 18))
            with pytest.raises(h264r.H264RError) as e:
                dec.check()
        finally:
            dec.set_debug(0)
        assert e.value.status == A.EDEVICE, flag


def test_gpu_ippp_chain_yuv_compare(L, dec, tmp_path):
    """Output/compare step over a dependent IPPP chain: each decoded
    picture is kept as reference slot 0 of the next (picture_end keep_slot); the GPU's
    frames are written cropped (output.cc:109-227) and compared per frame with the
    oracle's by the harness protocol (model/__init__.py:119-183)."""
    from h264r import output as OUT
    W, H, n = 22, 18, 4
    cfg = synth.default_cfg(L, 3, W, H)
    refs = synth.refpics(L, cfg)
    crop = OUT.Crop(left=1, right=2, top=0, bottom=4)
    gpu_yuv, want = tmp_path / "gpu.yuv", []
    oracle_refs = list(refs)
    with OUT.YuvWriter(gpu_yuv, W, H, crop) as w:
        for i in range(n):
            p = synth.picture(L, cfg, i)
            out = dec.decode_picture(p, refs if i == 0 else None, keep_slot=0)
            w.write(*out)
            ref_out = O.decode(p, oracle_refs)
            oracle_refs = [ref_out] + oracle_refs[1:]
            want.append(hashlib.md5(OUT.frame_bytes(*ref_out, w.geom)).hexdigest())
    OUT.write_digests(tmp_path / "gpu.yuv.md5", want)
    assert OUT.compare_yuv(gpu_yuv, tmp_path / "gpu.yuv.md5", "ippp") == want
    assert gpu_yuv.stat().st_size == n * w.geom.frame_bytes


def test_gpu_batch_latency_chain(L, dec):
    """bench.py's latency mode: a dependent chain through h264r_decode_batch, one picture
    per launch, each writing straight into the DPB slot the next one predicts from;
    the chain is compared with the oracle's (the same function bench.py times)."""
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    cfg = synth.default_cfg(L, 3, 22, 18)
    refs = synth.refpics(L, cfg)
    ms, n, ok = bench.latency_chain(dec, L, cfg, refs, torch.cuda.current_stream().cuda_stream, 4, 4)
    assert n == 4 and ms > 0
    assert ok is True


def test_gpu_expired_wait_reports_edevice(L, dec):
    """Every device-side wait is bounded in wall time (device_common.h wait_give_up): under
    H264R_DBG_WAIT_TEST every intra-walk wait asks for progress that never comes (10 ms
    bound); the launch drains, h264r_picture_end reports H264R_EDEVICE within that bound
    plus the drain, and the context decodes bit-exact again afterwards."""
    import time
    cfg = synth.default_cfg(L, 2, 22, 18)                 # all-intra: every row waits on the one above
    p = synth.picture(L, cfg, 0)
    refs = synth.refpics(L, cfg)
    want = O.decode(p, refs)
    for flag in (A.DBG_DEBLOCK_MB, A.DBG_DEBLOCK_ROWS):
        t0 = time.time()
        with pytest.raises(h264r.H264RError) as e:
            dec.decode_picture(p, refs, debug=A.DBG_WAIT_TEST | flag)
        assert e.value.status == A.EDEVICE
        assert time.time() - t0 < 5.0
        got = dec.decode_picture(p, refs, debug=flag)
        for k in range(3):
            assert np.array_equal(got[k], want[k]), (flag, k)


def test_gpu_async_pictures_overlap(L, dec):
    """h264r_picture_end_async / h264r_picture_wait: picture i+1 is staged and enqueued while
    picture i is still on the GPU, referencing the DPB slot picture i is written into (stream
    order); every picture equals the oracle's, the waits hand them out oldest first, a third
    picture before a wait and a synchronous end with pictures outstanding are H264R_ESTATE."""
    from h264r.mbview import iter_mbs
    W, H, n = 22, 18, 5
    cfg = synth.default_cfg(L, 3, W, H)
    refs = synth.refpics(L, cfg)
    for s, (y, u, v) in enumerate(refs):
        dec.set_ref(s, y, u, v)
    pics = [synth.picture(L, cfg, i) for i in range(n)]
    want, oracle_refs = [], list(refs)
    for p in pics:
        out = O.decode(p, oracle_refs)
        oracle_refs = [out] + oracle_refs[1:]
        want.append(out)

    def stage(p):
        dec.init(W, H, p.pic, p.slices)
        for addr, rec, lv, mv, rr in iter_mbs(p):
            dec.decode(addr, rec, lv, mv, rr)

    got = []
    stage(pics[0])
    dec.deblock_filter_async(keep_slot=0)
    for i in range(1, n):
        stage(pics[i])
        dec.deblock_filter_async(keep_slot=0)
        if i == 2:
            with pytest.raises(h264r.H264RError) as e:
                dec.init(W, H, pics[0].pic, pics[0].slices)     # two pictures outstanding
            assert e.value.status == A.ESTATE
        got.append(dec.wait())
    with pytest.raises(h264r.H264RError) as e:
        stage(pics[0])
        dec.deblock_filter()                                   # one picture outstanding
    assert e.value.status == A.ESTATE
    got.append(dec.wait())
    for i in range(n):
        for k in range(3):
            d = first_diff(got[i][k], want[i][k], 16 if k == 0 else 8)
            assert d is None, f"picture {i} plane {k}: {d}"
