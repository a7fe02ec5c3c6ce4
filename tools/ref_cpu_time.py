#!/usr/bin/env python3
"""Time the compiled, unmodified reference decoder (oracle/_ref/ref_driver, built from
/root/reference by `make -C oracle ref`) on the bench workloads, one thread, same seeded
synthetic pictures as bench.py -- the cross-check BASELINE.md section 4 asks for.  This
container only (the GPU box has no reference sources).  Each timed run reconstructs one
picture `reps` times (ref_driver.cc timing mode: coefficient push, Decoder::decode of
every MB, deblock_filter); its output is checked against the oracle.

    python tools/ref_cpu_time.py --out profiles/r02_reference_cpu.json
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "arrow-h264_amd")]

import numpy as np  # noqa: E402

import _oracle as O  # noqa: E402
from h264r import synth  # noqa: E402

SIZES = {2: (120, 68), 3: (120, 68), 4: (120, 68), 5: (240, 135)}


def cpu_model() -> str:
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            return line.split(":", 1)[1].strip()
    return "unknown"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,3,4,5")
    ap.add_argument("--pictures", type=int, default=3, help="distinct pictures per config")
    ap.add_argument("--seconds", type=float, default=4.0, help="target CPU seconds per picture")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    L = O.lib()
    res = {"what": "unmodified reference (luuvish/arrow-h264 decoder.cc path) compiled -O2, one thread, "
                   "post-entropy reconstruction: coefficient push + decode(mb) + deblock_filter",
           "cpu": cpu_model(), "configs": {}}
    for cidx in [int(c) for c in a.configs.split(",")]:
        W, H = SIZES[cidx]
        cfg = synth.default_cfg(L, cidx, W, H)
        refs = synth.refpics(L, cfg)
        mbs, sec = 0, 0.0
        for i in range(a.pictures):
            _, m1, s1 = O.run_reference(cfg, i, time_reps=1)
            reps = max(1, int(a.seconds / max(s1, 1e-6)))
            planes, m, s = O.run_reference(cfg, i, time_reps=reps)
            want = O.decode(synth.picture(L, cfg, i), refs)
            assert all(np.array_equal(x, y) for x, y in zip(planes, want)), f"config {cidx} picture {i}"
            mbs += m
            sec += s
        res["configs"][str(cidx)] = {"width_mbs": W, "height_mbs": H, "pictures": a.pictures,
                                     "macroblocks": mbs, "seconds": round(sec, 3),
                                     "macroblocks_per_s": round(mbs / sec, 1), "verified_vs_oracle": True}
        print(cidx, res["configs"][str(cidx)], flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    main()
