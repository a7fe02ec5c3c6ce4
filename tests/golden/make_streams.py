"""Regenerate the stream-level parity fixtures (this container only: needs /root/reference).

For every stream of tests/streams.py STREAMS:
  1. write it with the repo's bitstream writer (tests/h264_writer.py) into
     tests/golden/streams/<name>.264;
  2. decode it with the UNMODIFIED reference decoder (oracle/_ref/ldecod, compiled from
     /root/reference by `make -C oracle ref`) and record the per-frame MD5s of its YUV
     (the reference harness's protocol, script/test/model/__init__.py:119-183);
  3. decode it with the reference parser + drop-in Decoder shim over the CPU oracle
     (oracle/_ref/ldecod_shim) under H264R_CAPTURE, check that its YUV has the same
     per-frame MD5s, and save what crossed the C ABI as <name>.cap.npz.

    make -C oracle ref && python tests/golden/make_streams.py [name ...]

With names, only those streams are (re)generated; the other entries of streams.json stay.
"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import h264_writer as W  # noqa: E402
import streams as S  # noqa: E402

from h264r import output as OUT  # noqa: E402

REF = os.path.join(S.ROOT, "oracle", "_ref")


def decode(binary: str, stream: str, out: str, env=None) -> str:
    r = subprocess.run([os.path.join(REF, binary), "-i", stream, "-o", out], capture_output=True, text=True,
                       timeout=600, env=env, cwd=os.path.dirname(out))
    if r.returncode != 0:
        raise RuntimeError(f"{binary} {stream}: rc {r.returncode}\n{r.stdout[-1500:]}\n{r.stderr[-1500:]}")
    return r.stdout


def main() -> None:
    os.makedirs(S.STREAM_DIR, exist_ok=True)
    only = set(sys.argv[1:])
    unknown = only - set(S.STREAMS)
    if unknown:
        raise SystemExit(f"no such streams: {sorted(unknown)}")
    table = json.load(open(S.STREAMS_JSON))["streams"] if only and os.path.exists(S.STREAMS_JSON) else {}
    for name, cfg in S.STREAMS.items():
        if only and name not in only:
            continue
        data = W.write_stream(S.stream_path(name), W.StreamCfg(**cfg))
        with tempfile.TemporaryDirectory() as td:
            ref_yuv, shim_yuv, cap = (os.path.join(td, f) for f in ("ref.yuv", "shim.yuv", "cap.bin"))
            decode("ldecod", S.stream_path(name), ref_yuv)
            decode("ldecod_shim", S.stream_path(name), shim_yuv, env=dict(os.environ, H264R_CAPTURE=cap))
            want = OUT.digest_by_frames(ref_yuv, cfg["frames"])
            got = OUT.digest_by_frames(shim_yuv, cfg["frames"])
            if got != want:
                raise SystemExit(f"{name}: reference parser + shim differs from the reference: {got} vs {want}")
            pics = S.read_capture_file(cap)
            nfr = len(pics) - sum(1 for p in pics if S.structure(p) in (1, 2)) // 2   # a field pair is one frame
            if nfr != cfg["frames"]:
                raise SystemExit(f"{name}: captured {len(pics)} pictures, {nfr} frames for {cfg['frames']}")
            S.save_capture(S.capture_path(name), pics)
        table[name] = {"cfg": cfg, "bytes": len(data), "frame_md5": want,
                       "source": "oracle/_ref/ldecod (unmodified reference) per-frame MD5 of the cropped YUV"}
        print(f"{name}: {len(data)} bytes, {cfg['frames']} frames, shim == reference")
    table = {n: table[n] for n in S.STREAMS if n in table}          # the order of STREAMS
    with open(S.STREAMS_JSON, "w") as f:
        json.dump({"streams": table}, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
