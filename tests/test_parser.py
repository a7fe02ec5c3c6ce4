"""The repo's own CPU entropy / syntax stage (include/h264p.h,
arrow-h264_amd/parser/h264p.cc).

The parser replaces the reference's parser (interpret_*.cc, slice_*.cc, dpb.cc) on the
caller side of the reconstruction ABI.  It is pinned two ways on the committed writer
streams (tests/streams.py):

* its decode reproduces the UNMODIFIED reference's per-frame MD5s (tests/golden/streams.json)
  -- on the CPU implementation of the h264r ABI here (oracle/_cpu/h264dec_cpu), and on
  MI355X through libh264r.so (arrow-h264_amd/lib/h264dec);
* what it hands the ABI is byte-identical to what the reference parser + drop-in shim handed
  it (the committed captures, tests/golden/streams/*.cap.npz): every MB record, level block,
  motion entry, slice table, picture record, quantisation table and DPB slot.

Both entropy coders are covered: 16 CAVLC streams (I / P / B / SP, lossless, long-term
references) and 5 CABAC streams (every cabac_init_idc, I_PCM inside CABAC slices, B
pictures with 8x8 transforms, BASELINE config 4's 1080p High IBBP 4-slice shape).
"""
import os
import subprocess

import numpy as np
import pytest

import _oracle as O
import streams as S
from h264r import output as OUT

GOLD = S.golden()["streams"]
NAMES = [n for n in S.STREAMS if n not in S.PARSER_REFUSED]
CPU_DEC = os.path.join(S.ROOT, "oracle", "_cpu", "h264dec_cpu")
GPU_DEC = os.path.join(S.ROOT, "arrow-h264_amd", "lib", "h264dec")


def _cpu_dec():
    O.build_oracle()
    assert os.path.exists(CPU_DEC)
    return CPU_DEC


def _run(binary, name, out, env=None):
    return subprocess.run([binary, "-i", S.stream_path(name), "-o", str(out)], capture_output=True, text=True,
                          timeout=600, env=dict(os.environ, **(env or {})))


@pytest.mark.parametrize("name", NAMES)
def test_parser_decodes_to_reference_md5s(name, tmp_path):
    """Own parser + the CPU implementation of the reconstruction ABI == the unmodified
    reference decoder, frame by frame (the reference harness's protocol,
    script/test/model/__init__.py:119-183)."""
    out = tmp_path / "out.yuv"
    r = _run(_cpu_dec(), name, out)
    assert r.returncode == 0, r.stderr[-800:]
    assert OUT.digest_by_frames(str(out), S.STREAMS[name]["frames"]) == GOLD[name]["frame_md5"]


@pytest.mark.parametrize("name", NAMES)
def test_parser_hands_the_abi_what_the_reference_parser_did(name, tmp_path):
    """Every array the parser passes through the C ABI equals the capture of the reference
    parser + shim (the same h264r_picture_begin / h264r_mb_submit / h264r_picture_end
    traffic, in the same order, with the same DPB slots)."""
    cap = tmp_path / "cap.bin"
    r = _run(_cpu_dec(), name, tmp_path / "out.yuv", {"H264R_CAPTURE": str(cap)})
    assert r.returncode == 0, r.stderr[-800:]
    mine = S.read_capture_file(str(cap))
    ref = S.load_capture(S.capture_path(name))
    assert len(mine) == len(ref)
    for i, (a, b) in enumerate(zip(mine, ref)):
        assert a["keep"] == b["keep"], f"picture {i}: DPB slot"
        for k in ("mbs", "levels", "mv", "ref_idx", "slices", "pic", "quant"):
            if a[k].dtype.names:
                for f in a[k].dtype.names:
                    assert np.array_equal(a[k][f], b[k][f]), f"picture {i}: {k}.{f}"
            else:
                assert np.array_equal(a[k], b[k]), f"picture {i}: {k}"
        assert a["plane_md5"] == b["plane_md5"], f"picture {i}: reconstructed planes"


@pytest.mark.parametrize("name", ["bp_qcif_ippp", "hp_cif_cabac_ibbp_4slices"])
def test_parser_synchronous_mode_matches(name, tmp_path):
    """H264P_SYNC=1 (h264r_picture_end per picture instead of the overlapped
    h264r_picture_end_async / h264r_picture_wait pair): the same frames."""
    out = tmp_path / "out.yuv"
    r = _run(_cpu_dec(), name, out, {"H264P_SYNC": "1"})
    assert r.returncode == 0, r.stderr[-800:]
    assert OUT.digest_by_frames(str(out), S.STREAMS[name]["frames"]) == GOLD[name]["frame_md5"]


@pytest.mark.parametrize("name", [n for n in NAMES if "slices" in n])
def test_parser_parallel_slices_hand_the_abi_the_same(name, tmp_path):
    """The slices of a picture parsed on 4 threads (H264P_THREADS=4): the ABI traffic and the
    frames are those of the sequential parse, i.e. the reference parser + shim's."""
    cap = tmp_path / "cap.bin"
    out = tmp_path / "out.yuv"
    r = _run(_cpu_dec(), name, out, {"H264R_CAPTURE": str(cap), "H264P_THREADS": "4"})
    assert r.returncode == 0, r.stderr[-800:]
    assert OUT.digest_by_frames(str(out), S.STREAMS[name]["frames"]) == GOLD[name]["frame_md5"]
    mine = S.read_capture_file(str(cap))
    ref = S.load_capture(S.capture_path(name))
    assert len(mine) == len(ref)
    for i, (a, b) in enumerate(zip(mine, ref)):
        for k in ("mbs", "levels", "mv", "ref_idx", "slices", "pic", "quant"):
            if a[k].dtype.names:
                for f in a[k].dtype.names:
                    assert np.array_equal(a[k][f], b[k][f]), f"picture {i}: {k}.{f}"
            else:
                assert np.array_equal(a[k], b[k]), f"picture {i}: {k}"


def test_parser_covers_both_entropy_coders():
    assert {bool(c.get("cabac")) for c in S.STREAMS.values()} == {False, True}


def test_parser_rejects_garbage(tmp_path):
    """A stream whose slice names no PPS, and a truncated slice: errors, not crashes."""
    bad = tmp_path / "bad.264"
    bad.write_bytes(bytes([0, 0, 0, 1, 0x65, 0x88, 0x84, 0x00]))
    r = subprocess.run([_cpu_dec(), "-i", str(bad), "-o", str(tmp_path / "o.yuv")], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode != 0 and "h264dec:" in r.stderr
    data = open(S.stream_path("bp_qcif_ippp"), "rb").read()
    cut = tmp_path / "cut.264"
    cut.write_bytes(data[: len(data) // 3])
    r = subprocess.run([_cpu_dec(), "-i", str(cut), "-o", str(tmp_path / "o.yuv")], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode != 0 and "h264dec:" in r.stderr


# ---------------------------------------------------------------------------- MI355X
@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_parser_decodes_to_reference_md5s(name, tmp_path):
    """The standalone decoder of the GPU box (no reference code anywhere): own parser +
    libh264r.so on MI355X reproduces the unmodified reference's per-frame MD5s."""
    assert os.path.exists(GPU_DEC), "arrow-h264_amd/lib/h264dec not built"
    out = tmp_path / "out.yuv"
    r = _run(GPU_DEC, name, out)
    assert r.returncode == 0, r.stderr[-800:]
    assert OUT.digest_by_frames(str(out), S.STREAMS[name]["frames"]) == GOLD[name]["frame_md5"]


def _decode_bytes(binary, data: bytes, tmp_path, tag: str, timeout=120):
    src = tmp_path / f"{tag}.264"
    src.write_bytes(data)
    out = tmp_path / f"{tag}.yuv"
    r = subprocess.run([binary, "-i", str(src), "-o", str(out)], capture_output=True, text=True, timeout=timeout)
    return r, (out.read_bytes() if out.exists() else b"")


@pytest.mark.parametrize("names", [("bp_qcif_ippp", "bp_cif_wp_pcm"), ("bp_cif_wp_pcm", "bp_qcif_ippp"),
                                   ("hp_cif_cabac_ibbp_4slices", "bp_qcif_longterm_40", "hp_720p_4slices")])
def test_parser_resolution_change_at_idr(names, tmp_path):
    """Streams of different picture sizes back to back (every one opens with its SPS / PPS, ids 0,
    and an IDR): the decode is each stream's own decode in turn -- a replaced active SPS ends the
    open picture first (slice_header.cc:392-423), the picture still on the device leaves the
    context at its own size, and every output frame keeps its own size and cropping
    (a resolution decrease overflowed the host copy, an increase lost a picture)."""
    dec = _cpu_dec()
    whole, parts = b"", []
    for n in names:
        data = open(S.stream_path(n), "rb").read()
        whole += data
        r, y = _decode_bytes(dec, data, tmp_path, n)
        assert r.returncode == 0, r.stderr[-800:]
        parts.append(y)
    r, y = _decode_bytes(dec, whole, tmp_path, "all")
    assert r.returncode == 0, r.stderr[-800:]
    assert y == b"".join(parts)


def test_parser_malformed_streams_under_asan(tmp_path):
    """Malformed headers and slice data (bytes of the committed streams flipped at random, seeded)
    through the parser built with AddressSanitizer + UBSan: every run ends in a decoded stream or
    a reported error, never an out-of-bounds access or undefined behaviour (ue(v)
    values >= 2^31 turned negative in int fields, unbounded list modifications, unchecked SPS /
    slice-header ranges)."""
    O.build_oracle()
    subprocess.run(["make", "-s", "-C", os.path.join(S.ROOT, "oracle"), "asan"], check=True)
    asan = os.path.join(S.ROOT, "oracle", "_cpu", "h264dec_cpu_asan")
    rng = np.random.default_rng(0x264A)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    bad = []
    for name in ("bp_qcif_ippp", "mp_qcif_ibbp_direct", "hp_qcif_cabac_intra_qp0_51", "hp_qcif_scaling_lists",
                 "hp_qcif_ibbp_explicit_8x8", "xp_qcif_sp", "bp_qcif_slices_cip", "hi444_qcif_lossless"):
        base = bytearray(open(S.stream_path(name), "rb").read())
        for k in range(60):
            data = bytearray(base)
            # the first bytes hold SPS / PPS / the first slice header; later flips hit MB data
            for _ in range(int(rng.integers(1, 4))):
                pos = int(rng.integers(4, min(len(data), 96))) if k % 2 == 0 else int(rng.integers(4, len(data)))
                data[pos] ^= 1 << int(rng.integers(0, 8))
            if k % 6 == 5:
                # an oversized ue(v) in a parameter set or the first slice header: 32 (k % 12 == 5) or
                # 40 zero bits then a one, i.e. RBSP 00 00 00 00 [00] 80 with its emulation-prevention
                # bytes (an RBSP 00 00 0x with x <= 3 is sent as 00 00 03 0x), so that Bits::ue() sees
                # 32+ leading zeros (values >= 2^31: ue_max / se_in reject them)
                pos = int(rng.integers(8, 40))
                data[pos:pos + 4] = (b"\x00\x00\x03\x00\x00\x80" if k % 12 == 5 else b"\x00\x00\x03\x00\x00\x03\x00\x80")
            src = tmp_path / f"{name}_{k}.264"
            src.write_bytes(bytes(data))
            r = subprocess.run([asan, "-i", str(src), "-o", str(tmp_path / "o.yuv")], capture_output=True, text=True,
                               timeout=120, env=env)
            if "Sanitizer" in r.stderr or "runtime error" in r.stderr or r.returncode < 0:
                bad.append((name, k, r.returncode, r.stderr[-1500:]))
    assert not bad, bad[0]


def test_parser_oversized_ue_rejected_under_asan(tmp_path):
    """ue(v) codes of 31, 32 and 40 leading zero bits (values from 2^31 - 1 up: past every int
    field) reach Bits::ue() through emulation-prevention bytes in an SPS (seq_parameter_set_id),
    and the ASan + UBSan build reports an error for each, with no sanitizer message."""
    O.build_oracle()
    subprocess.run(["make", "-s", "-C", os.path.join(S.ROOT, "oracle"), "asan"], check=True)
    asan = os.path.join(S.ROOT, "oracle", "_cpu", "h264dec_cpu_asan")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    head = b"\x00\x00\x00\x01\x67\x42\x00\x1e"          # start code, SPS NAL, Baseline, level 3.0
    codes = {31: b"\x00\x00\x03\x00\x01\xff\xff\xff\xfe",     # RBSP 00 00 00 01 ff ff ff fe
             32: b"\x00\x00\x03\x00\x00\x80",                  # RBSP 00 00 00 00 80
             40: b"\x00\x00\x03\x00\x00\x03\x00\x80"}          # RBSP 00 00 00 00 00 80
    for zeros, body in codes.items():
        src = tmp_path / f"ue{zeros}.264"
        src.write_bytes(head + body)
        r = subprocess.run([asan, "-i", str(src), "-o", str(tmp_path / "o.yuv")], capture_output=True, text=True,
                           timeout=60, env=env)
        assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-1500:]
        assert r.returncode > 0 and "h264dec:" in r.stderr, (zeros, r.returncode, r.stderr[-500:])


@pytest.mark.parametrize("name", sorted(S.PARSER_REFUSED))
def test_parser_refuses_what_it_does_not_reproduce(name, tmp_path):
    """The streams the own parser does not yet decode like the reference are refused with a
    message naming the feature, never decoded wrongly (their shim captures still replay on the GPU)."""
    r = _run(_cpu_dec(), name, tmp_path / "out.yuv")
    assert r.returncode != 0 and S.PARSER_REFUSED[name] in r.stderr, r.stderr[-400:]
