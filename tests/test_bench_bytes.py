"""bench.py's roofline numerator: the per-kernel algorithmic bytes (kernel_bytes) split
the SURVEY 8(d) per-MB total (h264r_synth_algo_bytes) exactly between the inter and
intra kernels, and k_deblock's share is 768 B per MB (every sample read and written once)."""
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
    assert inter + intra == total
    assert deblock == 3 * 11 * 9 * 768
    assert (intra > 0) and (cidx == 2 or inter > 0)
