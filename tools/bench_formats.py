"""Throughput of the chroma formats on the reconstruction path (off the headline metric): the
config-3 workload (1080p P pictures) generated in 4:2:0, 4:2:2, 4:4:4 and 4:0:0 and as
4:2:0 MBAFF frames (H264R_FORMATS=mbaff,1,... selects), one
h264r_decode_batch of B pictures per step, timed with HIP events on the launch stream over K
steps after W warm-up steps; picture 0 of each format checked against the oracle first.

    python3 tools/bench_formats.py [B] [K] [W]
    rocprofv3 --kernel-trace --stats -d gpurun_out/fmt -o fmt -- python3 tools/bench_formats.py

One JSON line per format: {"chroma_format", "pictures", "ms_per_step", "macroblocks_per_s",
"verified_vs_oracle"}.  TEST / MEASUREMENT TOOL: it loads the oracle (tests/_oracle.py) as the
checker only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "arrow-h264_amd"))


def main():
    import numpy as np
    import torch
    import _oracle as O
    import h264r
    from h264r import batch as B
    from h264r import synth
    npics = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    warm = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    L = h264r.lib()
    from h264r import _abi as A
    W, H = 120, 68
    only = os.environ.get("H264R_FORMATS")            # e.g. "mbaff" or "1,2"
    fmts = [f if f == "mbaff" else int(f) for f in only.split(",")] if only else [1, 2, 3, 0, "mbaff"]
    for fmt in fmts:
        # "mbaff": the config-3 workload as MBAFF frames (4:2:0, frame / field MB pairs)
        mb = fmt == "mbaff"
        cfg = synth.default_cfg(L, 3, W, H, **(dict(structure=A.MBAFF_FRAME) if mb else
                                              dict(chroma_format=fmt if fmt else A.SYNTH_CHROMA_400)))
        fmt = 1 if mb else fmt
        pics = [synth.picture(L, cfg, i % 8) for i in range(npics)]
        refs = synth.refpics(L, cfg)
        dec = h264r.Decoder(0, W, H, chroma_format=fmt)
        for s, (y, u, v) in enumerate(refs):
            dec.set_ref(s, y, u, v)
        db = B.to_device(B.pack(pics, h264r.quant_flat()), npics, None)
        stream = torch.cuda.current_stream()
        sp = stream.cuda_stream
        dec.decode_batch(db.batch, stream=sp)
        dec.check()
        want = O.decode(pics[0], refs)
        got = db.planes(0)
        ok = all(np.array_equal(got[k], want[k]) for k in range(3 if fmt else 1))
        for _ in range(warm):
            dec.decode_batch(db.batch, stream=sp)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record(stream)
        for _ in range(steps):
            dec.decode_batch(db.batch, stream=sp)
        b.record(stream)
        torch.cuda.synchronize()
        dec.check()
        ms = a.elapsed_time(b) / steps
        print(json.dumps({"chroma_format": fmt, "workload": "1080p P pictures (config 3)" + (", MBAFF frames" if mb else ""),
                          "pictures": npics,
                          "ms_per_step": ms, "macroblocks_per_s": npics * W * H / (ms / 1e3),
                          "verified_vs_oracle": ok}), flush=True)
        dec.close()
        del db


if __name__ == "__main__":
    main()
