"""Regenerate tests/golden/cabac_tables.json (this container only: needs /root/reference).

What the CABAC side of the repo's bitstream writer (tests/h264_writer.py) encodes with, as
the reference decoder has it (oracle/probe_cabac.cc):

* init: per slice kind (I; P and B with cabac_init_idc 0..2) and context (the reference's
  own context layout, cabac_contexts_t bitstream_cabac.h:61-83) the (m, n) pair that
  reproduces the probed initial (pStateIdx, valMPS) at every SliceQpY 0..51 through
  preCtxState = clip3(1, 126, ((m * QP) >> 4) + n) (9.3.1.1); null where the reference
  leaves a context uninitialised for that slice kind;
* the engine tables rangeTabLPS / transIdxLPS / transIdxMPS (black-box decode_decision);
* the residual context maps of residual_block_cabac.

    make -C oracle ref && python tests/golden/make_cabac_tables.py
"""
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
QP = np.arange(52)


def pre_state(v):
    """preCtxState of a probed (pStateIdx | valMPS << 6)."""
    s, mps = v & 63, v >> 6
    return s + 64 if mps else 63 - s


def fit(pre):
    """(m, n) with clip3(1, 126, ((m * QP) >> 4) + n) == pre for every QP."""
    m = np.arange(-128, 128)[:, None]
    n_cands = [int(pre[0])] if 1 < pre[0] < 126 else (list(range(-128, 2)) if pre[0] == 1 else list(range(126, 128)))
    for n in n_cands:
        got = np.clip(((m * QP[None, :]) >> 4) + n, 1, 126)
        ok = np.nonzero((got == pre[None, :]).all(axis=1))[0]
        if len(ok):
            return int(m[ok[0], 0]), n
    raise SystemExit("cabac: no (m, n) reproduces a probed context")


def main():
    out = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "probe_cabac")], check=True,
                         capture_output=True, text=True).stdout
    d = json.loads(out)
    init = {}
    for key, rows in d["init"].items():
        a = np.array(rows)                               # [qp][ctx]
        mn = []
        for k in range(a.shape[1]):
            col = a[:, k]
            if (col == 255).all():
                mn.append(None)
                continue
            pre = np.array([pre_state(int(v)) for v in col])
            mn.append(list(fit(pre)))
        init[key] = mn
    d["init"] = init
    # the field scans (Tables 8-13 / 8-14, field) as the reference maps scan positions of a field
    # picture: Transform::inverse_scan_luma_ac on a field slice (oracle/ref_driver.cc)
    scans = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "ref_driver"), "11", "4", "0", "1", "0", "0", "0",
                            "1", "0", "0", "0", "20", "30", "0", "0", "4", "4", "1", "0", "/dev/null", "0", "0",
                            "0", "1"], check=True, capture_output=True, text=True,
                           env=dict(os.environ, H264R_PRINT_FIELD_SCANS="1")).stdout
    d.update(json.loads(scans))
    d["_source"] = ("oracle/probe_cabac.cc: cabac_contexts_t::init (bitstream_cabac.cc:1215-1264) called for every "
                    "slice kind / cabac_init_idc / SliceQpY, fitted to (m, n) per context; engine tables from "
                    "cabac_engine_t::decode_decision (interpret.cc:318-341) as a black box; residual context maps "
                    "of residual_block_cabac (interpret_residual.cc:175-270)")
    with open(os.path.join(HERE, "cabac_tables.json"), "w") as f:
        json.dump(d, f, separators=(",", ":"))
        f.write("\n")
    print("cabac_tables.json:", sum(v is not None for v in init["P0"]), "P contexts,",
          sum(v is not None for v in init["I"]), "I contexts")


if __name__ == "__main__":
    main()
