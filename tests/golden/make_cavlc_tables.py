"""Regenerate tests/golden/cavlc_tables.json (this container only: needs /root/reference).

The CAVLC code tables of H.264 (Tables 9-5, 9-7..9-9, 9-10) as the reference decoder
reads them, derived by oracle/probe_cavlc.cc, which feeds every 16-bit pattern to the
reference's own coeff_token / total_zeros / run_before readers
(interpret_se.cc:606-674) and records value -> (length, code).  The repo's bitstream
writer (tests/h264_writer.py) encodes with these tables.

    make -C oracle ref && python tests/golden/make_cavlc_tables.py
"""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def main():
    out = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "probe_cavlc")], check=True,
                         capture_output=True, text=True).stdout
    d = json.loads(out)
    d["_source"] = ("oracle/probe_cavlc.cc: the reference's VLC readers (interpret_se.cc:606-674) run on every "
                    "16-bit pattern; coeff_token entries [TotalCoeff, TrailingOnes, length, code] per nC class, "
                    "total_zeros [value, length, code] per (table yuv, tzVlcIndex), run_before per zerosLeft")
    with open(os.path.join(HERE, "cavlc_tables.json"), "w") as f:
        json.dump(d, f, separators=(",", ":"))
        f.write("\n")


if __name__ == "__main__":
    main()
