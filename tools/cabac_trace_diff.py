"""tools/cabac_trace_diff.py <StreamCfg as JSON> -- debug the bitstream writer: write the
stream, decode it with the reference parser's syntax-element trace (oracle/_ref/ldecod_trace,
this container only) and print the first syntax element where the parser and the writer's
own log (h264_cabac.CabacSink) part ways, with the context before it."""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import h264_writer as W  # noqa: E402


def main():
    cfg = W.StreamCfg(**json.loads(sys.argv[1]))
    enc = W.Encoder(cfg)
    enc.se_log = []
    data = enc.stream()
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "s.264")
        open(path, "wb").write(data)
        r = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "ldecod_trace"), "-i", path, "-o", os.devnull],
                           capture_output=True, text=True, cwd=td, timeout=300)
    got = [l[3:] for l in r.stderr.splitlines() if l.startswith("SE ")]
    want = enc.se_log
    for i, (g, w) in enumerate(zip(got, want)):
        if g != w:
            print(f"first difference at syntax element {i}: parser '{g}' writer '{w}'")
            for k in range(max(0, i - 12), min(len(want), i + 3)):
                print(f"  {k:6d} parser {got[k] if k < len(got) else '-':40s} writer {want[k]}")
            return 1
    print(f"{min(len(got), len(want))} syntax elements agree (parser {len(got)}, writer {len(want)})")
    return 0


if __name__ == "__main__":
    sys.exit(main())
