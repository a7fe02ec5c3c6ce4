"""Debug helper (GPU box): decode small batches with the row-walk deblocking kernel and
list where the planes differ from the oracle (plane, MB x, MB y, row in MB)."""
import sys, os, collections
sys.path[:0] = ["tests", "arrow-h264_amd"]
import numpy as np
import _oracle as O
import h264r
from h264r import _abi as A, batch as B, synth

L = O.lib()
def run(W, H, n, cidx=3, **over):
    cfg = synth.default_cfg(L, cidx, W, H, **over)
    pics = [synth.picture(L, cfg, i) for i in range(n)]
    refs = synth.refpics(L, cfg)
    want = [O.decode(p, refs) for p in pics]
    with h264r.Decoder(0, W, H) as dec:
        for s, (y, u, v) in enumerate(refs):
            dec.set_ref(s, y, u, v)
        host = B.pack(pics, h264r.quant_flat())
        db = B.to_device(host, n, None)
        dec.set_debug(A.DBG_DEBLOCK_ROWS)
        dec.decode_batch(db.batch)
        dec.check()
        bad = collections.Counter()
        npic = 0
        for i in range(n):
            got = db.planes(i)
            anyb = False
            for k in range(3):
                m = 16 if k == 0 else 8
                for (yy, xx) in np.argwhere(got[k] != want[i][k]):
                    bad[(k, xx // m, yy // m, yy % m)] += 1
                    anyb = True
            npic += anyb
    print(f"W={W} H={H} n={n} cidx={cidx} {over}: bad pictures {npic}, (plane, mbx, mby, row) top: {bad.most_common(12)}", flush=True)

for args in [(11, 9, 33), (11, 9, 16), (11, 9, 1), (12, 9, 16), (11, 8, 16), (22, 18, 16)]:
    run(*args, pcm_permille=20)
