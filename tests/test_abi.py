"""C-ABI library: loads, exports every symbol include/h264r.h declares, struct
layouts agree between C and the numpy/ctypes mirror, host helpers agree with the
oracle.  No compute calls (no GPU needed)."""
import ctypes as C
import os
import re
import subprocess
import sys
import tempfile

import numpy as np
import pytest

import _oracle as O
import h264r
from h264r import _abi as A

ROOT = O.ROOT


@pytest.fixture(scope="module")
def L():
    h264r.build()
    return h264r.lib()


def header_symbols(name):
    txt = open(os.path.join(ROOT, "include", name)).read()
    return sorted(set(re.findall(r"\b(h264r_\w+)\s*\(", txt)))


@pytest.mark.parametrize("hdr", ["h264r.h", "h264r_synth.h", "h264r_group.h"])
def test_exports_every_declared_symbol(L, hdr):
    syms = header_symbols(hdr)
    assert len(syms) >= 5
    for s in syms:
        assert hasattr(L, s), f"{s} declared in include/{hdr} but not exported"


def test_struct_layouts_match_c():
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "h264r.h"
#include "h264r_synth.h"
#include "h264r_group.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu\n", sizeof(h264r_mb), sizeof(h264r_slice), sizeof(h264r_quant),
         sizeof(h264r_pic), sizeof(h264r_batch), sizeof(h264r_synth_cfg));
  printf("%zu %zu %zu %zu\n", offsetof(h264r_mb, coef_off), offsetof(h264r_mb, ipred),
         offsetof(h264r_slice, ref_slot), offsetof(h264r_slice, implicit_w1));
  printf("%zu %zu %zu\n", offsetof(h264r_batch, ref_planes), offsetof(h264r_synth_cfg, seed),
         offsetof(h264r_batch, ref_planes_stride));
  printf("%zu %zu\n", sizeof(h264r_transport), offsetof(h264r_transport, finish));
  return 0; }
'''
    with tempfile.TemporaryDirectory() as td:
        c = os.path.join(td, "l.c")
        open(c, "w").write(src)
        exe = os.path.join(td, "l")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()
    v = [int(x) for x in out]
    assert v[0:6] == [A.MB_DTYPE.itemsize, A.SLICE_DTYPE.itemsize, A.QUANT_DTYPE.itemsize,
                      A.PIC_DTYPE.itemsize, C.sizeof(A.Batch), C.sizeof(A.SynthCfg)]
    assert v[6:10] == [A.MB_DTYPE.fields["coef_off"][1], A.MB_DTYPE.fields["ipred"][1],
                       A.SLICE_DTYPE.fields["ref_slot"][1], A.SLICE_DTYPE.fields["implicit_w1"][1]]
    assert v[10:13] == [A.Batch.ref_planes.offset, A.SynthCfg.seed.offset, A.Batch.ref_planes_stride.offset]
    from h264r import group as G
    assert v[13:15] == [C.sizeof(G.Transport), G.Transport.finish.offset]


def test_quant_flat_matches_oracle(L):
    assert np.array_equal(h264r.quant_flat().view(np.uint8), O.quant_flat().view(np.uint8))


def test_quant_lists_flat_equals_flat(L):
    flat4 = (C.c_int32 * 16)(*([16] * 16))
    flat8 = (C.c_int32 * 64)(*([16] * 64))
    arr = (C.c_void_p * 12)(*([C.cast(flat4, C.c_void_p)] * 6 + [C.cast(flat8, C.c_void_p)] * 6))
    q = np.zeros(1, A.QUANT_DTYPE)
    assert L.h264r_quant_init_lists(A.ptr(q), arr) == 0
    assert np.array_equal(q.view(np.uint8), h264r.quant_flat().view(np.uint8))


def test_error_codes(L):
    assert L.h264r_abi_version() == A.ABI_VERSION
    assert L.h264r_strerror(A.EINVAL) == b"invalid argument"
    h = C.c_void_p()
    assert L.h264r_create(C.byref(h), 0, 0, 0, 1, 8) == A.EINVAL
    assert L.h264r_create(C.byref(h), 0, 10, 10, 4, 8) == A.EUNSUPPORTED     # no chroma_format_idc 4
    assert L.h264r_create(C.byref(h), 0, 10, 10, 1, 10) == A.EUNSUPPORTED
    assert L.h264r_quant_init_flat(None) == A.EINVAL
    assert L.h264r_destroy(None) == A.EINVAL
    assert L.h264r_mb_submit(None, 0, None, None, 0, None, None) == A.EINVAL


def test_no_gpu_means_no_decoder(L):
    """Without a gfx950 device the product refuses to run (no CPU fallback)."""
    if L.h264r_device_count() > 0:
        pytest.skip("a GPU is present")
    h = C.c_void_p()
    assert L.h264r_create(C.byref(h), 0, 10, 10, 1, 8) == A.ENODEVICE
    with pytest.raises(h264r.H264RError):
        h264r.Decoder()
    # a group over device planes needs the device too (host planes: device -1, test_dist.py)
    from h264r import group as G
    with pytest.raises(h264r.H264RError):
        G.Group(2, 0, 0, "torch")


@pytest.mark.parametrize("env", [{"H264R_DEBLOCK2_MIN": "abc"}, {"H264R_LEVELS": "99"}, {"H264R_COOP": "2"},
                                 {"H264R_DEBUG": "1"}, {"H264R_WAIT_MS": "0"}])
def test_env_knob_out_of_range_is_refused(env):
    """Every environment knob of the library is validated once: a value outside its range makes
    h264r_create fail with H264R_EINVAL (before any device query, so this runs without a GPU)
    instead of being taken for another setting.  H264R_DEBUG may carry
    schedule flags only: DBG_NO_DEBLOCK (1) would change the output."""
    code = ("import ctypes as C, sys; sys.path.insert(0, %r); import h264r; L = h264r.lib(); h = C.c_void_p(); "
            "print(L.h264r_create(C.byref(h), 0, 10, 10, 1, 8))" % os.path.join(ROOT, "arrow-h264_amd"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, **env))
    assert r.returncode == 0, r.stderr[-1000:]
    assert int(r.stdout.split()[-1]) == A.EINVAL
    assert list(env)[0] in r.stderr
