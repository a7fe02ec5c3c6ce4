#!/usr/bin/env python3
"""tools/isa_dpp.py -- the DPP instruction forms in libh264r.so's gfx950 code objects.

The kernels exchange values between lanes with DPP moves (device_common.h lane_xor1 /
lane_xor4 / lane_lo4 / lane_hi4 / quad_bcast), and the compiler may fold a DPP move into the
VOP2 instruction that consumes it (GCNDPPCombine: v_add_u32_dpp, v_and_b32_dpp, ...).  On MI355X
a reversed VOP2 opcode with DPP (v_subrev_u32_dpp, v_lshlrev_b32_dpp) applies the lane select to
src1 instead of src0 (tools/dpp/dpp_fold_test.hip); round 5's wrong residuals were the lane ^ 1
low / high moves folded into v_subrev_u32_dpp.  This tool lists every (mnemonic, DPP modifiers)
pair in the built library so that tests/test_isa.py can refuse reversed opcodes and hold the rest
to the verified set -- a toolchain or source change that produces a new form fails at build time
instead of waiting for a GPU parity run.

    python tools/isa_dpp.py [path/to/libh264r.so]
"""
from __future__ import annotations

import collections
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(path: str, arch: str = "gfx950") -> list[bytes]:
    """The device code objects of every offload bundle embedded in a host ELF (the
    clang-offload-bundler layout: magic, entry count, then {offset, size, triple} per entry,
    offsets relative to the bundle start)."""
    data = open(path, "rb").read()
    out, pos = [], 0
    while True:
        i = data.find(MAGIC, pos)
        if i < 0:
            return out
        off = i + len(MAGIC)
        (n,) = struct.unpack_from("<Q", data, off)
        off += 8
        for _ in range(n):
            eo, es, ts = struct.unpack_from("<QQQ", data, off)
            off += 24
            triple = data[off:off + ts].decode()
            off += ts
            if arch in triple and es:
                out.append(data[i + eo:i + eo + es])
        pos = i + len(MAGIC)


def dpp_forms(path: str) -> collections.Counter:
    """Counter of (kernel, mnemonic, modifiers) over every DPP instruction."""
    forms: collections.Counter = collections.Counter()
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(code_objects(path)):
            f = os.path.join(td, f"co{k}.o")
            open(f, "wb").write(co)
            asm = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", f], check=True, capture_output=True,
                                 text=True).stdout
            kern = None
            for ln in asm.splitlines():
                m = re.match(r"^[0-9a-f]+ <(\w+)>:", ln)
                if m:
                    kern = m.group(1)
                if "_dpp" not in ln:
                    continue
                toks = ln.split("//")[0].split()
                mods = " ".join(t for t in toks[1:] if ":" in t)
                forms[(kern, toks[0], mods)] += 1
    return forms


def main() -> int:
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "arrow-h264_amd", "lib", "libh264r.so")
    for (kern, op, mods), n in sorted(dpp_forms(path).items()):
        print(f"{n:4d}  {kern:16s} {op:18s} {mods}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
