"""bench.py's roofline numerator: the per-kernel algorithmic bytes (kernel_bytes) partition
the SURVEY 8(d) total (h264r_synth_algo_bytes) with no byte counted twice: the MBs' R
between the inter and intra kernels, their W (384 B per MB) to deblocking."""
import os
import sys

import pytest

from h264r import synth
import h264r

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


@pytest.mark.parametrize("cidx", [2, 3, 4])
def test_kernel_bytes_partition_the_algorithmic_total(cidx):
    L = h264r.lib()
    cfg = synth.default_cfg(L, cidx, 11, 9)
    pics = [synth.picture(L, cfg, i) for i in range(3)]
    total = sum(sum(synth.algo_bytes(L, p)) for p in pics)
    inter, intra, deblock = bench.kernel_bytes(pics, 11 * 9)
    assert inter + intra + deblock == total
    assert deblock == 3 * 11 * 9 * 384
    assert (intra > 0) and (cidx == 2 or inter > 0)
