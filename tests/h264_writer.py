"""h264_writer -- the repo's own tiny H.264 bitstream writer (TEST INFRASTRUCTURE).

SURVEY.md 8(c) item 2: the conformance streams the reference's harness decodes are not
in the container, so stream-level parity is pinned on streams this module generates.
It writes Annex-B byte streams (CAVLC only) that exercise the reconstruction path:

* SPS (Baseline 66 or High 100 with CAVLC), PPS, IDR + P pictures, several slices per
  picture, per-slice deblocking control (disable_deblocking_filter_idc 0/1/2, alpha/beta
  offsets), chroma_qp_index_offset, constrained_intra_pred, frame cropping, multiple
  reference frames, explicit weighted prediction;
* macroblocks I_PCM, I_16x16 (4 modes, every CBP), I_4x4 (9 modes, predicted-mode
  coding), I_8x8 (High: transform_size_8x8_flag), P_L0_16x16 / 16x8 / 8x16 / 8x8 (all
  sub-partitions) and P_8x8ref0, P_Skip runs, intra MBs in P slices, mb_qp_delta;
* CAVLC residuals (coeff_token / levels with suffix-length adaptation and escapes /
  total_zeros / run_before) for luma DC/AC/4x4/8x8 (interleaved) and chroma DC/AC, with
  the decoder's nC prediction from neighbouring blocks.

The encoder never needs the reconstruction: motion vector differences and QP deltas are
drawn at random and the decoder derives the rest.  Intra modes are drawn only among
those the neighbour availability allows (the reference asserts otherwise,
intra_prediction.cc:191-873), and the predicted intra mode is derived exactly as the
decoder does (neighbour.cc:318-360) so the chosen mode is what gets decoded.

The VLC tables come from tests/golden/cavlc_tables.json, probed from the reference's
own readers (oracle/probe_cavlc.cc).  Syntax follows the reference parser:
slice header interpret_rbsp.cc:625-765, MB layer interpret_mb.cc:180-316 and 506-744,
residual interpret_residual.cc:64-174 and 421-494.
"""
from __future__ import annotations

import json
import os
import random
from dataclasses import dataclass, field

import h264_cabac as CB

HERE = os.path.dirname(os.path.abspath(__file__))
_T = json.load(open(os.path.join(HERE, "golden", "cavlc_tables.json")))

COEFF_TOKEN = {int(nc): {(tc, t1): (ln, code) for tc, t1, ln, code in ent} for nc, ent in _T["coeff_token"].items()}
TOTAL_ZEROS = {int(y): {int(t): {v: (ln, code) for v, ln, code in ent} for t, ent in d.items()}
               for y, d in _T["total_zeros"].items()}
RUN_BEFORE = {int(z): {v: (ln, code) for v, ln, code in ent} for z, ent in _T["run_before"].items()}
CBP_CODE = {k: {cbp: code for code, cbp in enumerate(v)} for k, v in _T["cbp_me"].items()}
# chroma_format_idc 0 / 3: the other half of Table 9-4 (no chroma CBP)
CBP_CODE_444 = {k: {cbp: code for code, cbp in enumerate(v)} for k, v in _T["cbp_me_444"].items()}

# 4x4 / 8x8 frame zig-zag scans: raster index of scan position k (spec Tables 8-12/8-13)
def _zigzag(n):
    out = []
    for s in range(2 * n - 1):
        cells = [(s - x, x) for x in range(n) if 0 <= s - x < n]    # (y, x) along the anti-diagonal
        cells = sorted(cells, key=lambda c: c[1]) if s % 2 else sorted(cells, key=lambda c: -c[1])
        out += [y * n + x for y, x in cells]
    return out


ZZ4 = _zigzag(4)
ZZ8 = _zigzag(8)

SKIP, INTER, I4, I8, I16, PCM = range(6)


class BitWriter:
    def __init__(self):
        self.bits: list[int] = []

    def u(self, n: int, v: int) -> None:
        for k in range(n - 1, -1, -1):
            self.bits.append((v >> k) & 1)

    def ue(self, v: int) -> None:
        v += 1
        nb = v.bit_length() - 1
        self.u(nb, 0)
        self.u(nb + 1, v)

    def se(self, v: int) -> None:
        self.ue(2 * v - 1 if v > 0 else -2 * v)

    def code(self, lc) -> None:
        self.u(lc[0], lc[1])

    def aligned(self) -> bool:
        return len(self.bits) % 8 == 0

    def trailing(self) -> None:
        self.bits.append(1)
        while len(self.bits) % 8:
            self.bits.append(0)

    def bytes(self) -> bytes:
        assert len(self.bits) % 8 == 0
        return bytes(int("".join(map(str, self.bits[i:i + 8])), 2) for i in range(0, len(self.bits), 8))


def nal_unit(ref_idc: int, typ: int, rbsp: bytes) -> bytes:
    """Annex-B NAL unit: start code, header, emulation-prevention bytes (7.4.1)."""
    out = bytearray([0, 0, 0, 1, (ref_idc << 5) | typ])
    zeros = 0
    for b in rbsp:
        if zeros >= 2 and b <= 3:
            out.append(3)
            zeros = 0
        out.append(b)
        zeros = zeros + 1 if b == 0 else 0
    return bytes(out)


@dataclass
class StreamCfg:
    width_mbs: int = 11
    height_mbs: int = 9
    frames: int = 4
    seed: int = 1
    profile: int = 66                # 66 Baseline, 88 Extended, 100 High, 244 High 4:4:4 Predictive (4:2:0, CAVLC)
    num_refs: int = 1                # max_num_ref_frames
    slices: int = 1                  # slices per picture (random first_mb_in_slice)
    qp: tuple = (18, 38)
    chroma_qp_offset: int = 0
    second_chroma_qp_offset: int | None = None
    cip: int = 0                     # constrained_intra_pred_flag
    deblock: tuple = (0,)            # disable_deblocking_filter_idc choices per slice
    offsets: int = 0                 # max |alpha/beta offset_div2|
    crop: tuple = (0, 0, 0, 0)       # left, right, top, bottom (luma samples / 2)
    weighted: int = 0                # weighted_pred_flag (explicit WP in P slices)
    transform8x8: int = 0            # High: transform_8x8_mode_flag
    pcm: float = 0.02
    skip: float = 0.15
    intra_in_p: float = 0.10
    level_max: int = 6               # typical |level|; escapes drawn now and then
    all_intra: bool = False          # every picture an IDR / I picture
    mv_range: int = 24               # |mvd| bound (quarter samples)
    scaling: int = 0                 # High: 1 SPS scaling matrix, 2 PPS matrix, 3 both
    sp: float = 0.0                  # 88: share of P pictures coded as SP pictures (every slice SP)
    qs: tuple = (0, 5)               # QsY range of SP slices (the reference's itrans_sp_cr is defined for QsC < 6)
    lossless: float = 0.0            # 244: qpprime_y_zero_transform_bypass_flag; share of coded intra
                                     # MBs sent to QP 0 (TransformBypassModeFlag, interpret_mb.cc:804).
                                     # Coded inter MBs keep QP >= 1: the reference's inter bypass
                                     # reads stale Intra4x4PredMode (transform.cc:993)
    bframes: int = 0                 # B pictures between anchors (IBBP...; pic_order_cnt_type 0, B pictures
                                     # decoded after the anchor that follows them in output order)
    bipred: int = 0                  # weighted_bipred_idc: 0 default, 1 explicit, 2 implicit (POC distances)
    direct: tuple = (0, 1)           # direct_spatial_mv_pred_flag choices per B slice (0 temporal, 1 spatial)
    b_ref: float = 0.0               # share of B pictures kept as references (nal_ref_idc != 0)
    l1_refs: int = 2                 # max num_ref_idx_l1_active of B slices
    cabac: int = 0                   # entropy_coding_mode_flag (CABAC, tests/h264_cabac.py; Main / High)
    cabac_init: tuple = (0, 1, 2)    # cabac_init_idc choices per P / B slice
    field: float = 0.0               # > 0: frame_mbs_only_flag 0 and this share of the frames coded as two
                                     # field pictures (PAFF: field_pic_flag, the second field in the
                                     # first's frame; 1.0 = every frame); P fields predict from any
                                     # reference field (the first field of their own frame too)
    bottom_first: float = 0.0        # share of field pairs sent bottom field first
    mbaff: float = 0.0               # > 0: MBAFF frames (frame_mbs_only_flag 0, mb_adaptive_frame_field_flag 1),
                                     # this share of the MB pairs field pairs (mb_field_decoding_flag); CAVLC,
                                     # no CIP, I and P pictures.  A pair whose two MBs are skipped takes the
                                     # inferred flag (the left pair's, else the upper pair's, else frame); a
                                     # pair whose top MB alone is skipped codes the flag in its bottom MB
    chroma_format: int = 1           # chroma_format_idc (profiles 100 / 122 / 244): 1 4:2:0, 2 4:2:2 (CAVLC:
                                     # 8 chroma 4x4 blocks and a 2x4 DC per plane, nC -2, interpret_residual.cc:462-494),
                                     # 3 4:4:4 (244, CAVLC: Cb and Cr coded as luma, residual_luma per plane
                                     # interpret_residual.cc:497-505; no intra chroma mode, the 4:4:4 CBP table),
                                     # 0 4:0:0 (100 / 122 / 244: luma only -- no chroma mode, residual, PCM
                                     # samples or chroma weights; the ChromaArrayType 0 CBP table)
    long_term: int = 0               # the IDR is a long-term reference (LongTermFrameIdx 0) kept for the
                                     # whole stream, and P picture `long_term` becomes a second one by
                                     # MMCO 4 + 6 (LongTermFrameIdx 1); P pictures predict from them
                                     # (list 0: short-term by PicNum, then long-term, 8.2.4.2.1)


@dataclass
class _Mb:
    kind: int = SKIP
    slice: int = -1
    intra: bool = False
    fld: bool = False                # mb_field_decoding_flag (MBAFF frames)
    i4: list = field(default_factory=lambda: [2] * 16)   # Intra4x4PredMode, blkIdx order
    i8: list = field(default_factory=lambda: [2] * 4)
    t8: bool = False
    nz: list = field(default_factory=lambda: [[[0] * 4 for _ in range(4)] for _ in range(3)])
    # what the CABAC context selection reads of a decoded MB (mb_t fields, macroblock.h:78-135)
    skip: bool = False
    mbt_ref: int = 0                 # mb_t::mb_type (0 skip / direct, 1..4 partitions, 8 I_4x4, 9 I_8x8, 10 I_16x16, 12 I_PCM)
    cbpl: int = 0
    cbpc: int = 0
    cmode: int = 0
    cbp_bits: int = 0
    sub_direct: list = field(default_factory=lambda: [False] * 4)
    ref: list = field(default_factory=lambda: [[-1] * 16, [-1] * 16])
    mvd: list = field(default_factory=lambda: [[(0, 0)] * 16, [(0, 0)] * 16])


def _blk_xy(blk: int):
    """(x, y) in 4x4 units of luma4x4BlkIdx (6.4.3)."""
    return ((blk // 4) % 2) * 2 + (blk % 4) % 2, ((blk // 4) // 2) * 2 + (blk % 4) // 2


class Encoder:
    def __init__(self, cfg: StreamCfg):
        self.c = cfg
        self.rng = random.Random(cfg.seed)
        self.W, self.H = cfg.width_mbs, cfg.height_mbs
        self.FH = cfg.height_mbs                 # frame height; a field picture has FH / 2 MB rows
        assert not cfg.field or cfg.height_mbs % 2 == 0
        assert not cfg.mbaff or (cfg.height_mbs % 2 == 0 and not cfg.cip and not cfg.bframes and
                                 not cfg.field)
        self.log2_max_frame_num = 4
        self.log2_max_poc_lsb = 8
        self.cab = None                  # the CABAC sink of the slice being written (CABAC streams)

    # ------------------------------------------------------------------ parameter sets
    def sps(self) -> bytes:
        c, w = self.c, BitWriter()
        w.u(8, c.profile)
        w.u(8, 0)                                   # constraint flags
        w.u(8, 51)                                  # level_idc (largest DPB)
        w.ue(0)                                     # seq_parameter_set_id
        if c.profile in (100, 122, 244):
            w.ue(c.chroma_format)                   # chroma_format_idc
            if c.chroma_format == 3:
                w.u(1, 0)                           # separate_colour_plane_flag
            w.ue(0); w.ue(0)                        # bit depths 8
            w.u(1, 1 if c.lossless else 0)          # qpprime_y_zero_transform_bypass_flag
            w.u(1, c.scaling & 1)                   # seq_scaling_matrix_present_flag
            if c.scaling & 1:
                self._scaling_matrix(w, 12 if c.chroma_format == 3 else 8)
        w.ue(self.log2_max_frame_num - 4)
        if c.bframes:
            w.ue(0)                                 # pic_order_cnt_type 0: B pictures reorder
            w.ue(self.log2_max_poc_lsb - 4)
        else:
            w.ue(2)                                 # pic_order_cnt_type 2 (output = decode order)
        w.ue(c.num_refs)                            # max_num_ref_frames
        w.u(1, 0)                                   # gaps_in_frame_num_value_allowed_flag
        w.ue(self.W - 1)
        if c.field or c.mbaff:
            w.ue(self.FH // 2 - 1)                  # pic_height_in_map_units_minus1 (field MB rows)
            w.u(1, 0)                               # frame_mbs_only_flag
            w.u(1, 1 if c.mbaff else 0)             # mb_adaptive_frame_field_flag
        else:
            w.ue(self.H - 1)
            w.u(1, 1)                               # frame_mbs_only_flag
        w.u(1, 1)                                   # direct_8x8_inference_flag
        crop = any(c.crop)
        w.u(1, 1 if crop else 0)
        if crop:
            for v in c.crop:
                w.ue(v)
        w.u(1, 0)                                   # vui_parameters_present_flag
        w.trailing()
        return nal_unit(3, 7, w.bytes())

    def pps(self) -> bytes:
        c, w = self.c, BitWriter()
        w.ue(0); w.ue(0)
        w.u(1, c.cabac)                             # entropy_coding_mode_flag
        w.u(1, 0)                                   # bottom_field_pic_order_in_frame_present_flag
        w.ue(0)                                     # num_slice_groups_minus1
        w.ue(0); w.ue(0)                            # num_ref_idx_l0/l1_default_active_minus1
        w.u(1, c.weighted)                          # weighted_pred_flag
        w.u(2, c.bipred)                            # weighted_bipred_idc
        w.se(0); w.se(0)                            # pic_init_qp/qs_minus26
        w.se(c.chroma_qp_offset)
        w.u(1, 1)                                   # deblocking_filter_control_present_flag
        w.u(1, c.cip)
        w.u(1, 0)                                   # redundant_pic_cnt_present_flag
        if c.profile in (100, 122, 244):
            w.u(1, c.transform8x8)
            w.u(1, 1 if c.scaling & 2 else 0)       # pic_scaling_matrix_present_flag
            if c.scaling & 2:
                self._scaling_matrix(w, 6 + (6 if c.chroma_format == 3 else 2) * c.transform8x8)
            w.se(c.chroma_qp_offset if c.second_chroma_qp_offset is None else c.second_chroma_qp_offset)
        w.trailing()
        return nal_unit(3, 8, w.bytes())

    def _scaling_matrix(self, w: BitWriter, n: int) -> None:
        """scaling_list_present_flag + scaling_list() for n lists (7.3.2.1.1.1): absent
        (fall-back rules), "use default" (first delta makes nextScale 0), explicit values
        in zig-zag order, or explicit values cut short (nextScale 0 repeats the last)."""
        r = self.rng
        for i in range(n):
            kind = r.choice(["absent", "default", "explicit", "short"])
            w.u(1, 0 if kind == "absent" else 1)
            if kind == "absent":
                continue
            size = 16 if i < 6 else 64
            if kind == "default":
                w.se(-8)                            # nextScale = (8 - 8) % 256 = 0 at j = 0
                continue
            last = 8
            stop = r.randint(1, size - 1) if kind == "short" else size
            for j in range(size):
                if j == stop:
                    w.se((0 - last + 128) % 256 - 128)   # nextScale 0: the rest repeats `last`
                    break
                v = r.randint(4, 64)
                w.se((v - last + 128) % 256 - 128)
                last = v

    # ------------------------------------------------------------------ availability
    def _nbr(self, a: int, xN: int, yN: int, chroma: bool = False):
        """MBAFF frames: Neighbour::get_neighbour (neighbour.cc:123-173) of sample (xN, yN) of MB a
        (storage index: row 2 pair_row + bottom) -- the geometric frame sample, the MB holding it and
        the sample's place in that MB -- if decoded in the current slice: (mb, lx, ly) or None."""
        mw = mh = 8 if chroma else 16
        W = self.W
        mbx, mby = a % W, a // W
        m = self.mbs[a]
        lx = mbx * mw + xN
        ly = (mby >> 1) * 2 * mh + ((mby & 1) + 2 * yN if m.fld else (mby & 1) * mh + yN)
        if lx < 0 or lx >= W * mw or ly < 0 or ly >= self.H * mh:
            return None
        npy, nx, rr = ly // (2 * mh), lx // mw, ly % (2 * mh)
        top = self.mbs[2 * npy * W + nx]
        nb = (ly & 1) if top.fld else int(rr >= mh)
        nm = self.mbs[(2 * npy + nb) * W + nx]
        if nm.slice != m.slice:                          # other slice, or not decoded yet (slice -1)
            return None
        return nm, lx % mw, (rr // 2) if top.fld else rr % mh

    def _mb_at(self, x: int, y: int, cur_slice: int):
        if x < 0 or y < 0 or x >= self.W or y >= self.H:
            return None
        m = self.mbs[y * self.W + x]
        return m if m.slice == cur_slice else None

    def _intra_avail(self, x, y, s):
        """Availability for intra prediction (same slice, constrained_intra_pred)."""
        m = self._mb_at(x, y, s)
        if m is None or (self.c.cip and not m.intra):
            return None
        return m

    # ------------------------------------------------------------------ CAVLC residual
    def _nc(self, a: int, pl: int, bx: int, by: int, s: int) -> int:
        """nC of the block at (bx, by) (4x4 units, plane pl), neighbour.cc:263-314."""
        mx, my = a % self.W, a // self.W
        luma = pl == 0 or self.c.chroma_format == 3     # 4:4:4: Cb / Cr blocks in the luma grid
        nw = 4 if luma else 2                           # 4x4 blocks per MB: across, down
        nh = 4 if luma or self.c.chroma_format == 2 else 2
        if self.c.mbaff:                                # predict_nnz through get_neighbour
            def nz_at(dx, dy):
                n = self._nbr(a, bx * 4 + dx, by * 4 + dy, not luma)
                return None if n is None else n[0].nz[pl][n[2] // 4][n[1] // 4]
            na, nb = nz_at(-1, 0), nz_at(0, -1)
            if na is not None and nb is not None:
                return (na + nb + 1) >> 1
            return (na or 0) + (nb or 0)
        def nz_of(dx, dy):
            x, y = bx + dx, by + dy
            ox, oy = mx + (x // nw if x >= 0 else -1), my + (y // nh if y >= 0 else -1)
            if x >= 0 and y >= 0:
                return self.mbs[a].nz[pl][y][x]
            m = self._mb_at(ox, oy, s)
            if m is None:
                return None
            return m.nz[pl][y % nh][x % nw]
        na, nb = nz_of(-1, 0), nz_of(0, -1)
        if na is not None and nb is not None:
            return (na + nb + 1) >> 1
        return (na or 0) + (nb or 0)

    def _levels(self, n: int):
        """Random coefficient levels of one block (scan order, n coefficients)."""
        r = self.rng
        tc = min(n, int(r.expovariate(0.35))) if r.random() < 0.8 else r.randint(0, n)
        pos = sorted(r.sample(range(n), tc))
        out = [0] * n
        for p in pos:
            if r.random() < 0.03:
                v = r.randint(self.c.level_max, 60)
            else:
                v = 1 if r.random() < 0.55 else min(self.c.level_max, 1 + int(r.expovariate(0.6)))
            out[p] = v if r.random() < 0.5 else -v
        return out

    def _block(self, w: BitWriter, coeffs: list, nc: int, max_num: int) -> int:
        """residual_block_cavlc (9.2, interpret_residual.cc:64-174) of coefficients in
        scan order; returns TotalCoeff."""
        nzp = [k for k, v in enumerate(coeffs) if v]
        tc = len(nzp)
        lv = [coeffs[k] for k in nzp]                   # levelVal[0..tc-1], low to high frequency
        t1 = 0
        for v in reversed(lv):
            if abs(v) == 1 and t1 < 3:
                t1 += 1
            else:
                break
        if nc >= 8:
            w.u(6, 3 if tc == 0 else ((tc - 1) << 2) | t1)
        else:
            cls = -1 if nc == -1 else (-2 if nc == -2 else (0 if nc < 2 else (2 if nc < 4 else 4)))
            w.code(COEFF_TOKEN[cls][(tc, t1)])
        if tc == 0:
            return 0
        for k in range(tc - 1, tc - 1 - t1, -1):
            w.u(1, 1 if lv[k] < 0 else 0)
        suffix_len = 1 if tc > 10 and t1 < 3 else 0
        for k in range(tc - 1 - t1, -1, -1):
            v = lv[k]
            code = 2 * v - 2 if v > 0 else -2 * v - 1
            if k == tc - 1 - t1 and t1 < 3:
                code -= 2
            if suffix_len == 0:
                if code < 14:
                    w.u(code, 0); w.u(1, 1)
                elif code < 30:
                    w.u(14, 0); w.u(1, 1); w.u(4, code - 14)
                else:
                    assert code - 30 < 4096
                    w.u(15, 0); w.u(1, 1); w.u(12, code - 30)
            else:
                if code < (15 << suffix_len):
                    w.u(code >> suffix_len, 0); w.u(1, 1); w.u(suffix_len, code & ((1 << suffix_len) - 1))
                else:
                    assert code - (15 << suffix_len) < 4096
                    w.u(15, 0); w.u(1, 1); w.u(12, code - (15 << suffix_len))
            if suffix_len == 0:
                suffix_len = 1
            if abs(v) > (3 << (suffix_len - 1)) and suffix_len < 6:
                suffix_len += 1
        total_zeros = nzp[-1] + 1 - tc
        if tc < max_num:
            yuv = 0 if max_num == 4 else (1 if max_num == 8 else 2)
            w.code(TOTAL_ZEROS[yuv][tc][total_zeros])
        zl = total_zeros
        for k in range(tc - 1, 0, -1):
            if zl <= 0:
                break
            run = nzp[k] - nzp[k - 1] - 1
            w.code(RUN_BEFORE[min(zl, 7)][run])
            zl -= run
        return tc

    def _residual(self, w: BitWriter, a: int, m: _Mb, cbp: int, s: int) -> None:
        """residual_luma + residual_chroma (interpret_residual.cc:421-494)."""
        cbpl, cbpc = cbp & 15, cbp >> 4
        if self.cab:
            self._residual_cabac(m, cbpl, cbpc)
            return
        # residual_luma for Y, and for Cb and Cr in 4:4:4 (interpret_residual.cc:497-505)
        for pl in ((0, 1, 2) if self.c.chroma_format == 3 else (0,)):
            if m.kind == I16:
                self._block(w, self._levels(16), self._nc(a, pl, 0, 0, s), 16)
            for b8 in range(4):
                if m.t8 and (cbpl >> b8) & 1:
                    l8 = self._levels(64)
                    for b4 in range(4):
                        bx, by = _blk_xy(b8 * 4 + b4)
                        m.nz[pl][by][bx] = self._block(w, [l8[4 * k + b4] for k in range(16)], self._nc(a, pl, bx, by, s), 16)
                    continue
                for b4 in range(4):
                    bx, by = _blk_xy(b8 * 4 + b4)
                    if (cbpl >> b8) & 1:
                        if m.kind == I16:
                            m.nz[pl][by][bx] = self._block(w, self._levels(15), self._nc(a, pl, bx, by, s), 15)
                        else:
                            m.nz[pl][by][bx] = self._block(w, self._levels(16), self._nc(a, pl, bx, by, s), 16)
                    else:
                        m.nz[pl][by][bx] = 0
        if self.c.chroma_format in (0, 3):
            return
        nbc = 8 if self.c.chroma_format == 2 else 4     # chroma 4x4 blocks (= DC coefficients) per plane
        if cbpc & 3:
            for _pl in (1, 2):
                self._block(w, self._levels(nbc), -1 if nbc == 4 else -2, nbc)
        for pl in (1, 2):
            for b in range(nbc):
                bx, by = b % 2, b // 2
                if cbpc & 2:
                    m.nz[pl][by][bx] = self._block(w, self._levels(15), self._nc(a, pl, bx, by, s), 15)
                else:
                    m.nz[pl][by][bx] = 0

    def _residual_cabac(self, m: _Mb, cbpl: int, cbpc: int) -> None:
        """The same blocks and level draws as the CAVLC path, as residual_block_cabac calls:
        an 8x8 transform block is one 64-coefficient block (interpret_residual.cc:453-456)."""
        cab = self.cab
        assert self.c.chroma_format in (0, 1, 2), "CABAC streams: 4:0:0 / 4:2:0 / 4:2:2"   # (4:4:4: CAVLC)
        if m.kind == I16:
            cab.block(CB.LUMA_16DC, 0, 0, self._levels(16))
        for b8 in range(4):
            if not (cbpl >> b8) & 1:
                continue
            if m.t8:
                l8 = self._levels(64)
                if not any(l8):                  # no coded_block_flag for 8x8 blocks: >= 1 coefficient
                    l8[0] = 1
                cab.block(CB.LUMA_8x8, 0, b8 * 4, l8)
                continue
            for b4 in range(4):
                if m.kind == I16:
                    cab.block(CB.LUMA_16AC, 0, b8 * 4 + b4, self._levels(15))
                else:
                    cab.block(CB.LUMA_4x4, 0, b8 * 4 + b4, self._levels(16))
        if self.c.chroma_format == 0:
            return
        nbc = 8 if self.c.chroma_format == 2 else 4
        if cbpc & 3:
            for pl in (1, 2):
                cab.block(CB.CHROMA_DC, pl, 0, self._levels(nbc))
        if cbpc & 2:
            for pl in (1, 2):
                for b in range(nbc):
                    cab.block(CB.CHROMA_AC, pl, b, self._levels(15))

    # ------------------------------------------------------------------ intra modes
    def _pred_mode(self, a: int, m: _Mb, bx: int, by: int, s: int, n8: bool) -> int:
        """predIntra4x4PredMode / predIntra8x8PredMode (neighbour.cc:318-400)."""
        mx, my = a % self.W, a // self.W
        def mode_of(dx, dy):
            x, y = bx + dx, by + dy
            if self.c.mbaff:                             # get_neighbour of the sample (neighbour.cc:318-400)
                n = self._nbr(a, bx * 4 + (-1 if dx else 0), by * 4 + (-1 if dy else 0))
                if n is None:
                    return None
                nb, lx, ly = n[0], n[1] // 4, n[2] // 4
            elif x >= 0 and y >= 0:
                nb, lx, ly = m, x, y
            else:
                nb = self._intra_avail(mx + (-1 if x < 0 else 0), my + (-1 if y < 0 else 0), s)
                if nb is None:
                    return None
                lx, ly = x % 4, y % 4
            if nb.kind == I8:
                return nb.i8[(ly // 2) * 2 + lx // 2]
            if nb.kind == I4:
                blk = (ly // 2) * 8 + (lx // 2) * 4 + (ly % 2) * 2 + lx % 2
                return nb.i4[blk]
            return 2
        # the 4x4 blocks left of / above the block's top-left 4x4 (also for 8x8 blocks:
        # the reference looks at samples (x-1, y) and (x, y-1), neighbour.cc:367-391)
        ma, mb_ = mode_of(-1, 0), mode_of(0, -1)
        if ma is None or mb_ is None:
            return 2
        return min(ma, mb_)

    def _avail_abd(self, a: int, bx: int, by: int, n: int, s: int):
        """Availability of neighbours A, B, D of an n-wide block at (bx, by) (4x4 units)."""
        mx, my = a % self.W, a // self.W
        if self.c.mbaff:
            ok = lambda x, y: self._nbr(a, x, y) is not None
            return ok(bx * 4 - 1, by * 4), ok(bx * 4, by * 4 - 1), ok(bx * 4 - 1, by * 4 - 1)
        av = lambda dx, dy: self._intra_avail(mx + dx, my + dy, s) is not None
        A = bx > 0 or av(-1, 0)
        B = by > 0 or av(0, -1)
        if bx > 0 and by > 0:
            D = True
        elif bx == 0 and by > 0:
            D = av(-1, 0)
        elif bx > 0 and by == 0:
            D = av(0, -1)
        else:
            D = av(-1, -1)
        return A, B, D

    @staticmethod
    def _valid_nxn(A, B, D):
        need = {0: "B", 1: "A", 2: "", 3: "B", 4: "ABD", 5: "ABD", 6: "ABD", 7: "B", 8: "A"}
        have = {"A": A, "B": B, "D": D}
        return [md for md, req in need.items() if all(have[ch] for ch in req)]

    # ------------------------------------------------------------------ one macroblock
    def _mb(self, w: BitWriter, a: int, ptype: str, s: int, nref):
        """One macroblock: every random decision is drawn here in a fixed order; the syntax
        goes out as CAVLC bits into `w`, or as CABAC bins through self.cab (a CabacSink)
        when the stream is CABAC.  Returns False for a skipped MB."""
        c, r = self.c, self.rng
        cab = self.cab
        m = self.mbs[a]
        m.slice = s
        if cab:
            cab.start_mb(a)
        if c.mbaff:
            # mb_field_decoding_flag: both MBs' skip draws are made with the top MB (where the pair's
            # flag goes depends on them, interpret_mb.cc:208-262, slice_data.cc:505-523)
            W = self.W
            top = (a // W) % 2 == 0
            if top:
                self.pair_roll = (r.random(), r.random())
                sk = [ptype == "P" and x < c.skip for x in self.pair_roll]
                mx, py = a % W, (a // W) // 2            # inferred: left pair, else upper pair, else frame
                A = self.mbs[(2 * py) * W + mx - 1] if mx > 0 else None
                B = self.mbs[(2 * py - 1) * W + mx] if py > 0 else None
                inferred = A.fld if A is not None and A.slice == s else (B.fld if B is not None and B.slice == s else False)
                fld = inferred if (sk[0] and sk[1]) else r.random() < c.mbaff
                self.pair_skip = sk
                if cab:
                    # CABAC (interpret_mb.cc:186-262): the top MB's skip flag with the inferred flag; a
                    # skipped top MB reads the bottom MB's skip flag ahead (the bottom MB with the top MB's
                    # inferred flag) and then, for a coded bottom MB, the pair's flag
                    m.fld = inferred
                    if ptype != "I":
                        cab.skip_flag(sk[0])
                        if sk[0]:
                            m.skip = True
                            bm = self.mbs[a + W]
                            bm.slice, bm.fld = s, inferred
                            cab.start_mb(a + W)
                            cab.skip_flag(sk[1])
                            if not sk[1]:
                                cab.field_flag(fld)
                            cab.start_mb(a)
                    if not sk[0]:
                        cab.field_flag(fld)
                elif not sk[0]:
                    w.u(1, 1 if fld else 0)
                m.fld = fld
            else:
                m.fld = self.mbs[a - W].fld
                if cab:
                    if ptype != "I" and not self.pair_skip[0]:
                        cab.skip_flag(self.pair_skip[1])
                elif self.pair_skip[0] and not self.pair_skip[1]:
                    w.u(1, 1 if m.fld else 0)            # coded in the bottom MB after a skipped top MB
            roll = self.pair_roll[0 if top else 1]
        else:
            roll = r.random()
        if ptype in ("P", "B") and roll < c.skip:
            m.kind, m.intra, m.skip, m.mbt_ref = SKIP, False, True, 0
            m.nz = [[[0] * 4 for _ in range(4)] for _ in range(3)]
            if cab and not c.mbaff:
                cab.skip_flag(True)
            return False
        if cab and ptype != "I" and not c.mbaff:
            cab.skip_flag(False)
        intra = ptype == "I" or r.random() < c.intra_in_p
        base = 5 if ptype == "P" else (23 if ptype == "B" else 0)
        if intra:
            m.intra = True
            k = r.random()
            if k < c.pcm:
                m.kind = PCM
            elif k < 0.4:
                m.kind = I16
            elif c.transform8x8 and k < 0.7:
                m.kind = I8
            else:
                m.kind = I4
        else:
            m.intra = False
            m.kind = INTER
        mx, my = a % self.W, a // self.W
        A, B, D = self._avail_abd(a, 0, 0, 4, s)
        if m.kind == PCM:
            m.mbt_ref = 12
            npcm = 256 + {0: 0, 2: 256, 3: 512}.get(c.chroma_format, 128)   # 2 x MbWidthC x MbHeightC chroma samples
            if cab:
                cab.mb_type_intra(25)
                cab.pcm([r.randint(1, 255) for _ in range(npcm)])
            else:
                w.ue(base + 25)
                while not w.aligned():
                    w.u(1, 0)
                for _ in range(npcm):
                    w.u(8, r.randint(1, 255))
            m.nz = [[[16] * 4 for _ in range(4)] for _ in range(3)]
            return True
        cmodes = [0] + ([1] if A else []) + ([2] if B else []) + ([3] if A and B and D else [])
        if m.kind == I16:
            modes = ([0] if B else []) + ([1] if A else []) + [2] + ([3] if A and B and D else [])
            mode = r.choice(modes)
            cbpc = r.randint(0, 2) if c.chroma_format in (1, 2) else 0
            cbpl = 15 if r.random() < 0.5 else 0
            m.mbt_ref, m.cbpl, m.cbpc = 10, cbpl, cbpc
            cm = r.choice(cmodes)
            if cab:
                cab.mb_type_intra(1 + mode + 4 * cbpc + (12 if cbpl else 0))
                if c.chroma_format in (1, 2):
                    m.cmode = cm
                    cab.chroma_mode(cm)
            else:
                w.ue(base + 1 + mode + 4 * cbpc + (12 if cbpl else 0))
                if c.chroma_format in (1, 2):           # intra_chroma_pred_mode: ChromaArrayType 1 / 2 only
                    w.ue(cm)
            cbp = cbpl | cbpc << 4
        elif m.kind in (I4, I8):
            m.t8 = m.kind == I8
            m.mbt_ref = 9 if m.t8 else 8
            if cab:
                cab.mb_type_intra(0)
                if c.transform8x8:
                    cab.transform8x8(m.t8)
            else:
                w.ue(base + 0)
                if c.transform8x8:
                    w.u(1, 1 if m.t8 else 0)
            if m.kind == I4:
                for blk in range(16):
                    bx, by = _blk_xy(blk)
                    mode = r.choice(self._valid_nxn(*self._avail_abd(a, bx, by, 1, s)))
                    pred = self._pred_mode(a, m, bx, by, s, False)
                    m.i4[blk] = mode
                    if cab:
                        cab.intra_mode(mode, pred)
                    elif mode == pred:
                        w.u(1, 1)
                    else:
                        w.u(1, 0); w.u(3, mode if mode < pred else mode - 1)
            else:
                for b8 in range(4):
                    bx, by = (b8 % 2) * 2, (b8 // 2) * 2
                    mode = r.choice(self._valid_nxn(*self._avail_abd(a, bx, by, 2, s)))
                    pred = self._pred_mode(a, m, bx, by, s, True)
                    m.i8[b8] = mode
                    if cab:
                        cab.intra_mode(mode, pred)
                    elif mode == pred:
                        w.u(1, 1)
                    else:
                        w.u(1, 0); w.u(3, mode if mode < pred else mode - 1)
            cm = r.choice(cmodes)
            cbp = r.randint(0, 47) if c.chroma_format in (1, 2) else r.randint(0, 15)
            m.cbpl, m.cbpc = cbp & 15, cbp >> 4
            if cab:
                if c.chroma_format in (1, 2):
                    m.cmode = cm
                    cab.chroma_mode(cm)
                cab.cbp(cbp)
            elif c.chroma_format in (0, 3):
                w.ue(CBP_CODE_444["intra"][cbp])
            else:
                w.ue(cm)
                w.ue(CBP_CODE["intra"][cbp])
        elif ptype == "B":
            cbp, small = self._b_inter(w, nref, a)
            m.t8 = False
            if (cbp & 15) and c.transform8x8 and not small:
                m.t8 = r.random() < 0.5
                if cab:
                    cab.transform8x8(m.t8)
                else:
                    w.u(1, 1 if m.t8 else 0)
        else:
            mbt = r.choices([0, 1, 2, 3, 4], weights=[45, 12, 12, 21, 10])[0]
            if cab and mbt == 4:
                mbt = 3                                  # no P_8x8ref0 in CABAC (Table 9-37)
            m.mbt_ref = (1, 2, 3, 4, 4)[mbt]
            if cab:
                cab.mb_type_p(mbt)
            else:
                w.ue(mbt)
            parts = {0: [(0, 0, 4, 4)], 1: [(0, 0, 4, 2), (0, 2, 4, 2)], 2: [(0, 0, 2, 4), (2, 0, 2, 4)]}
            nr = nref * 2 if m.fld else nref            # a field MB's refIdx counts fields
            nhdr = nr
            def ref_idx(x0, y0, pw, ph):
                v = r.randrange(nr)
                if cab:
                    cab.ref_idx(v, nr, 0, x0, y0)
                    self._set_ref(m, 0, x0, y0, pw, ph, v)
                elif nhdr == 2:
                    w.u(1, 1 - v)
                elif nhdr > 2:
                    w.ue(v)
            def mvd(x0, y0, pw, ph):
                dx, dy = r.randint(-c.mv_range, c.mv_range), r.randint(-c.mv_range, c.mv_range)
                if cab:
                    cab.mvd(dx, 0, 0, x0, y0); cab.mvd(dy, 0, 1, x0, y0)
                    self._set_mvd(m, 0, x0, y0, pw, ph, (dx, dy))
                else:
                    w.se(dx); w.se(dy)
            small = False
            if mbt in (0, 1, 2):
                for p in parts[mbt]:
                    ref_idx(*p)
                for p in parts[mbt]:
                    mvd(*p)
            else:
                subs = [r.choice([0, 0, 1, 2, 3]) for _ in range(4)]
                small = any(sb != 0 for sb in subs)
                for sb in subs:
                    if cab:
                        cab.sub_p(sb)
                    else:
                        w.ue(sb)
                if mbt == 3:
                    for b8 in range(4):
                        ref_idx((b8 % 2) * 2, (b8 // 2) * 2, 2, 2)
                for b8, sb in enumerate(subs):
                    x8, y8 = (b8 % 2) * 2, (b8 // 2) * 2
                    for sp in {0: [(0, 0, 2, 2)], 1: [(0, 0, 2, 1), (0, 1, 2, 1)], 2: [(0, 0, 1, 2), (1, 0, 1, 2)],
                               3: [(0, 0, 1, 1), (1, 0, 1, 1), (0, 1, 1, 1), (1, 1, 1, 1)]}[sb]:
                        mvd(x8 + sp[0], y8 + sp[1], sp[2], sp[3])
            cbp = r.randint(0, 47) if c.chroma_format in (1, 2) else r.randint(0, 15)
            m.cbpl, m.cbpc = cbp & 15, cbp >> 4
            if cab:
                cab.cbp(cbp)
            else:
                w.ue((CBP_CODE_444 if c.chroma_format in (0, 3) else CBP_CODE)["inter"][cbp])
            m.t8 = False
            if (cbp & 15) and c.transform8x8 and not small:
                m.t8 = r.random() < 0.5
                if cab:
                    cab.transform8x8(m.t8)
                else:
                    w.u(1, 1 if m.t8 else 0)
        if cbp or m.kind == I16:
            lo, hi = c.qp
            if c.lossless and not m.intra:
                lo = max(lo, 1)
            target = 0 if (c.lossless and m.intra and r.random() < c.lossless) else r.randint(lo, hi)
            d = (target - self.qp_pred + 26) % 52 - 26
            if cab:
                cab.qp_delta(d)
            else:
                w.se(d)
            self.qp_pred = (self.qp_pred + d + 52) % 52
        self._residual(w, a, m, cbp, s)
        return True

    @staticmethod
    def _set_ref(m, lst, x0, y0, pw, ph, v):
        for y in range(y0, y0 + ph):
            for x in range(x0, x0 + pw):
                m.ref[lst][y * 4 + x] = v

    @staticmethod
    def _set_mvd(m, lst, x0, y0, pw, ph, v):
        for y in range(y0, y0 + ph):
            for x in range(x0, x0 + pw):
                m.mvd[lst][y * 4 + x] = v

    # B partitions: mb_type 1..21 -> prediction of partition 0 / 1 (Table 7-14); sub_mb_type
    # -> (prediction, sub-partitions) (Table 7-18); None = direct
    B_PARTS = {1: ("L0",), 2: ("L1",), 3: ("Bi",)}
    B_PARTS.update({4 + k: pr for k, pr in enumerate(
        [("L0", "L0")] * 2 + [("L1", "L1")] * 2 + [("L0", "L1")] * 2 + [("L1", "L0")] * 2 + [("L0", "Bi")] * 2 +
        [("L1", "Bi")] * 2 + [("Bi", "L0")] * 2 + [("Bi", "L1")] * 2 + [("Bi", "Bi")] * 2)})
    B_SUBS = {0: (None, 0), 1: ("L0", 1), 2: ("L1", 1), 3: ("Bi", 1), 4: ("L0", 2), 5: ("L0", 2), 6: ("L1", 2),
              7: ("L1", 2), 8: ("Bi", 2), 9: ("Bi", 2), 10: ("L0", 4), 11: ("L1", 4), 12: ("Bi", 4)}

    def _b_inter(self, w: BitWriter, nref: tuple, a: int):
        """An inter MB of a B slice (7.3.5.1-7.3.5.2; interpret_mb.cc:392-404, 480-503,
        636-700): mb_type B_Direct_16x16 / 16x16 / 16x8 / 8x16 / B_8x8 with direct and every
        sub-partition, then ref_idx of list 0, of list 1, mvd of list 0, of list 1 (CAVLC
        bits, or CABAC bins through self.cab).  Returns (cbp, has sub-partitions smaller
        than 8x8)."""
        c, r, cab = self.c, self.rng, self.cab
        m = self.mbs[a]
        n0, n1 = nref

        def ref_idx(n, lst, x0, y0, pw, ph):
            v = r.randrange(n)
            if cab:
                cab.ref_idx(v, n, lst, x0, y0)
                self._set_ref(m, lst, x0, y0, pw, ph, v)
            elif n == 2:
                w.u(1, 1 - v)
            elif n > 2:
                w.ue(v)

        def mvd(lst, x0, y0, pw, ph):
            dx, dy = r.randint(-c.mv_range, c.mv_range), r.randint(-c.mv_range, c.mv_range)
            if cab:
                cab.mvd(dx, lst, 0, x0, y0); cab.mvd(dy, lst, 1, x0, y0)
                self._set_mvd(m, lst, x0, y0, pw, ph, (dx, dy))
            else:
                w.se(dx); w.se(dy)
        k = r.random()
        mbt = 0 if k < 0.15 else (r.randint(1, 3) if k < 0.55 else (r.randint(4, 21) if k < 0.8 else 22))
        m.mbt_ref = 0 if mbt == 0 else (1 if mbt <= 3 else (4 if mbt == 22 else (2 if mbt % 2 == 0 else 3)))
        m.sub_direct = [mbt == 0] * 4
        if cab:
            cab.mb_type_b(mbt)
        else:
            w.ue(mbt)
        small = False
        if 1 <= mbt <= 21:
            preds = self.B_PARTS[mbt]
            geo = [(0, 0, 4, 4)] if mbt <= 3 else ([(0, 0, 4, 2), (0, 2, 4, 2)] if mbt % 2 == 0 else [(0, 0, 2, 4), (2, 0, 2, 4)])
            for lst, (name, n) in enumerate((("L0", n0), ("L1", n1))):
                for pr, g in zip(preds, geo):
                    if pr in (name, "Bi"):
                        ref_idx(n, lst, *g)
            for lst, name in enumerate(("L0", "L1")):
                for pr, g in zip(preds, geo):
                    if pr in (name, "Bi"):
                        mvd(lst, *g)
        elif mbt == 22:
            subs = [0 if r.random() < 0.3 else r.randint(1, 12) for _ in range(4)]
            small = any(self.B_SUBS[sb][1] > 1 for sb in subs)
            m.sub_direct = [sb == 0 for sb in subs]
            for sb in subs:
                if cab:
                    cab.sub_b(sb)
                else:
                    w.ue(sb)
            for lst, (name, n) in enumerate((("L0", n0), ("L1", n1))):
                for b8, sb in enumerate(subs):
                    if sb and self.B_SUBS[sb][0] in (name, "Bi"):
                        ref_idx(n, lst, (b8 % 2) * 2, (b8 // 2) * 2, 2, 2)
            for lst, name in enumerate(("L0", "L1")):
                for b8, sb in enumerate(subs):
                    if sb and self.B_SUBS[sb][0] in (name, "Bi"):
                        x8, y8 = (b8 % 2) * 2, (b8 // 2) * 2
                        nparts = self.B_SUBS[sb][1]
                        if nparts == 1:
                            sps = [(0, 0, 2, 2)]
                        elif nparts == 4:
                            sps = [(0, 0, 1, 1), (1, 0, 1, 1), (0, 1, 1, 1), (1, 1, 1, 1)]
                        elif sb in (4, 6, 8):            # 8x4
                            sps = [(0, 0, 2, 1), (0, 1, 2, 1)]
                        else:                            # 4x8
                            sps = [(0, 0, 1, 2), (1, 0, 1, 2)]
                        for sp in sps:
                            mvd(lst, x8 + sp[0], y8 + sp[1], sp[2], sp[3])
        cbp = r.randint(0, 47) if self.c.chroma_format in (1, 2) else r.randint(0, 15)
        m.cbpl, m.cbpc = cbp & 15, cbp >> 4
        if cab:
            cab.cbp(cbp)
        else:
            w.ue((CBP_CODE_444 if self.c.chroma_format in (0, 3) else CBP_CODE)["inter"][cbp])
        return cbp, small

    # ------------------------------------------------------------------ pictures
    def _pred_weight_table(self, w: BitWriter, nrefs: tuple, bi: bool) -> None:
        """pred_weight_table (7.3.3.2; interpret_rbsp.cc): per list and reference a luma and
        a chroma flag with weights / offsets.  For B slices the weights stay inside the
        bi-prediction constraint -128 <= w0 + w1 <= 128 (8.4.2.3)."""
        r = self.rng
        chroma = self.c.chroma_format != 0          # no chroma weights in 4:0:0 (7.3.3.2)
        ld, cd = r.randint(0, 7), r.randint(0, 7)
        w.ue(ld)
        if chroma:
            w.ue(cd)
        for n in nrefs:
            for _ in range(n):
                if r.random() < 0.7:
                    w.u(1, 1)
                    w.se(r.randint(-min(64, 1 << ld), min(127, 2 << ld)) if not bi else r.randint(-32, 64))
                    w.se(r.randint(-20, 20))
                else:
                    w.u(1, 0)
                if not chroma:
                    continue
                if r.random() < 0.7:
                    w.u(1, 1)
                    for _ in range(2):
                        w.se(r.randint(-min(64, 1 << cd), min(127, 2 << cd)) if not bi else r.randint(-32, 64))
                        w.se(r.randint(-20, 20))
                else:
                    w.u(1, 0)

    def picture(self, idx: int, idr: bool, kind: str | None = None, ref_idc: int = 3, poc: int = 0,
                structure: int = 0, second: bool = False, nref_field=0):
        """NAL units of picture idx: one per slice.  kind None = I (idr) or P; "B" writes a
        B picture (nal_ref_idc = ref_idc, POC lsb from poc).  structure 1 / 2: a top / bottom
        field picture (field_pic_flag, bottom_field_flag; FH / 2 MB rows), `second` the second
        field of its frame (same frame_num), `nref_field` its num_ref_idx_l0_active (a B field:
        the (l0, l1) pair)."""
        c, r = self.c, self.rng
        self.H = self.FH // 2 if structure else self.FH
        n = self.W * self.H
        self.mbs = [_Mb() for _ in range(n)]
        ptype = kind or ("I" if idr else "P")
        sp = ptype == "P" and c.sp > 0 and r.random() < c.sp   # (no draw otherwise: fixed streams stay)
        units = n // 2 if c.mbaff else n                  # MBAFF: first_mb_in_slice counts MB pairs
        starts = sorted({0} | set(r.sample(range(1, units), min(c.slices - 1, units - 1)))) if c.slices > 1 else [0]
        frame_num = 0 if idr else (self.frame_num + (0 if second else 1)) % (1 << self.log2_max_frame_num)
        tracked = bool(c.bframes or c.long_term)           # DPB bookkeeping of the IBBP / long-term streams
        if tracked and not idr:
            frame_num = (self.prev_ref_fn + 1) % (1 << self.log2_max_frame_num)
        if second:
            frame_num = self.frame_num                   # both fields of a frame share frame_num
        self.frame_num = frame_num
        if ref_idc:
            self.prev_ref_fn = frame_num
        avail = self.st + self.lt                            # reference frames in the DPB before this picture
        mmco_lt = c.long_term and ptype == "P" and idx == c.long_term
        if ptype == "B":
            nref_b = tuple(nref_field) if structure else (avail, min(avail, c.l1_refs))
        elif c.bframes:
            # a P picture leaves one reference out of its list: the pictures its motion
            # points to stay in the DPB for the B pictures' temporal direct (the co-located
            # reference must be in their list 0, 8.4.1.2.3)
            self.refs_p = max(1, min(avail, c.num_refs - 1))
        if not tracked:
            self.refs = 0 if idr else min(self.refs + 1, c.num_refs)
        out = []
        W = self.W
        # the MBs of a slice in decoding order (MBAFF: pair by pair, top then bottom, by storage index)
        order = (lambda f, e: [((q // 2) // W * 2 + q % 2) * W + (q // 2) % W for q in range(2 * f, 2 * e)]) \
            if c.mbaff else (lambda f, e: list(range(f, e)))
        for s, first in enumerate(starts):
            end = starts[s + 1] if s + 1 < len(starts) else units
            w = BitWriter()
            w.ue(first)
            w.ue(7 if ptype == "I" else (8 if sp else (6 if ptype == "B" else 5)))   # slice_type (all slices alike)
            w.ue(0)                                 # pic_parameter_set_id
            w.u(self.log2_max_frame_num, frame_num)
            if c.field or c.mbaff:
                w.u(1, 1 if structure else 0)       # field_pic_flag
                if structure:
                    w.u(1, 1 if structure == 2 else 0)   # bottom_field_flag
            if idr:
                w.ue(idx % 2)                       # idr_pic_id
            if c.bframes:
                w.u(self.log2_max_poc_lsb, poc % (1 << self.log2_max_poc_lsb))   # pic_order_cnt_lsb
            nref = self.refs if not tracked else (self.refs_p if c.bframes else avail)
            if structure and ptype != "B":
                nref = nref_field
            if ptype == "B":
                w.u(1, r.choice(c.direct))          # direct_spatial_mv_pred_flag
                w.u(1, 1)                           # num_ref_idx_active_override_flag
                w.ue(nref_b[0] - 1); w.ue(nref_b[1] - 1)
                w.u(1, 0); w.u(1, 0)                # ref_pic_list_modification_flag_l0 / _l1
                if c.bipred == 1:
                    self._pred_weight_table(w, nref_b, True)
            if ptype == "P":
                w.u(1, 1)                           # num_ref_idx_active_override_flag
                w.ue(nref - 1)
                w.u(1, 0)                           # ref_pic_list_modification_flag_l0
                if c.weighted:
                    ld, cd = r.randint(0, 7), r.randint(0, 7)
                    w.ue(ld)
                    if c.chroma_format != 0:
                        w.ue(cd)
                    for _ in range(nref):
                        if r.random() < 0.7:
                            w.u(1, 1); w.se(r.randint(-min(64, 1 << ld), min(127, 2 << ld))); w.se(r.randint(-20, 20))
                        else:
                            w.u(1, 0)
                        if c.chroma_format == 0:
                            continue
                        if r.random() < 0.7:
                            w.u(1, 1)
                            for _ in range(2):
                                w.se(r.randint(-min(64, 1 << cd), min(127, 2 << cd))); w.se(r.randint(-20, 20))
                        else:
                            w.u(1, 0)
            if idr:
                w.u(1, 0)                           # no_output_of_prior_pics_flag
                w.u(1, 1 if c.long_term else 0)     # long_term_reference_flag (LongTermFrameIdx 0)
            elif mmco_lt:
                w.u(1, 1)                           # adaptive_ref_pic_marking_mode_flag
                w.ue(4); w.ue(2)                    # MMCO 4: MaxLongTermFrameIdx = 1
                w.ue(6); w.ue(1)                    # MMCO 6: this picture long-term, LongTermFrameIdx 1
                w.ue(0)                             # end
            elif ref_idc:
                w.u(1, 0)                           # adaptive_ref_pic_marking_mode_flag
            init_idc = 0
            if c.cabac and ptype != "I":
                init_idc = r.choice(c.cabac_init)
                w.ue(init_idc)                      # cabac_init_idc
            lo, hi = c.qp
            sqp = r.randint(lo, hi)
            w.se(sqp - 26)
            self.qp_pred = sqp
            if sp:
                w.u(1, r.randint(0, 1))             # sp_for_switch_flag
                w.se(r.randint(*c.qs) - 26)         # slice_qs_delta (pic_init_qs 26)
            idc = r.choice(c.deblock)
            w.ue(idc)
            if idc != 1:
                w.se(r.randint(-c.offsets, c.offsets)); w.se(r.randint(-c.offsets, c.offsets))
            if c.cabac:
                while not w.aligned():
                    w.u(1, 1)                       # cabac_alignment_one_bit
                self.cab = CB.CabacSink(self, w.bits, ptype, sqp, init_idc, s, field=structure != 0)
                mbs = order(first, end)
                for k, a in enumerate(mbs):
                    self._mb(w, a, ptype, s, nref_b if ptype == "B" else nref)
                    if not c.mbaff or (a // W) % 2:       # MBAFF: after bottom MBs only (slice_data.cc:531)
                        self.cab.end_of_slice(k == len(mbs) - 1)   # the flush's last bit is rbsp_stop_one_bit
                self.cab = None
                while not w.aligned():
                    w.u(1, 0)                       # rbsp_alignment_zero_bit
            else:
                skip_run = 0
                for a in order(first, end):
                    coded = self._mb(w if ptype == "I" else _Deferred(w, skip_run), a, ptype, s,
                                     nref_b if ptype == "B" else nref)
                    if ptype != "I":
                        skip_run = 0 if coded else skip_run + 1
                if ptype != "I" and skip_run:
                    w.ue(skip_run)
                w.trailing()
            out.append(nal_unit(ref_idc, 5 if idr else 1, w.bytes()))
        if ref_idc and not second:                           # marking after the picture (8.2.5); a second
            if idr:                                          # field joins its first field's frame
                self.st, self.lt = (0, 1) if c.long_term else (1, 0)
            elif mmco_lt:
                self.lt += 1
            else:
                self.st = min(self.st + 1, c.num_refs - self.lt)   # sliding window: short-term only
        return out

    def stream(self) -> bytes:
        c = self.c
        out = [self.sps(), self.pps()]
        self.frame_num, self.refs, self.prev_ref_fn, self.st, self.lt = 0, 0, 0, 0, 0
        if c.field and c.bframes:
            return b"".join(out + self._field_stream_b())
        if c.field:
            return b"".join(out + self._field_stream())
        if not c.bframes:
            for i in range(c.frames):
                out += self.picture(i, idr=(i == 0 or c.all_intra))
            return b"".join(out)
        # IBBP: anchors (I / P) every bframes + 1 pictures in output order, each sent before
        # the B pictures that precede it; trailing pictures past the last anchor are P.
        # POC = 2 x output index (frames).
        order, k = [(0, None)], 0
        while k + 1 < c.frames:
            anchor = min(k + c.bframes + 1, c.frames - 1)
            order.append((anchor, None))
            order += [(b, "B") for b in range(k + 1, anchor)]
            k = anchor
        for i, (disp, kind) in enumerate(order):
            ref_idc = 3
            if kind == "B":
                ref_idc = 2 if self.rng.random() < c.b_ref else 0
            out += self.picture(i, idr=(i == 0), kind=kind, ref_idc=ref_idc, poc=2 * disp)
        return b"".join(out)


    def _field_stream(self) -> list:
        """PAFF, pic_order_cnt_type 2 (output = decoding order): each frame a frame picture
        or, with probability c.field, a pair of field pictures; every picture a reference.
        A field's list holds the reference FIELDS (8.2.4.2.5): two per reference frame in
        the DPB, and for the second field of a pair also the first field; the sliding window
        counts frames, and the first field's frame counts from when it is stored."""
        c, r = self.c, self.rng
        out, nfr = [], 0                        # reference frames in the DPB
        for i in range(c.frames):
            idr = i == 0 or c.all_intra
            fld = c.field >= 1.0 or r.random() < c.field
            if not fld:
                self.refs = max(nfr - 1, 0)         # picture() counts this frame's list as refs + 1
                out += self.picture(i, idr=idr)
                nfr = 1 if idr else min(nfr + 1, c.num_refs)
                continue
            first = 2 if c.bottom_first and r.random() < c.bottom_first else 1
            n1 = 0 if idr else min(2 * nfr, H264R_MAX_FIELD_REFS)
            out += self.picture(i, idr=idr, structure=first, nref_field=n1)
            nfr = 1 if idr else min(nfr + 1, c.num_refs)
            n2 = min(2 * (nfr - 1) + 1, H264R_MAX_FIELD_REFS)
            out += self.picture(i, idr=False, kind="I" if c.all_intra else "P", structure=3 - first,
                                second=True, nref_field=n2)
        return out


    def _field_stream_b(self) -> list:
        """IBBP with field pictures (pic_order_cnt_type 0): every frame a frame picture or,
        with probability c.field, a field pair; frame POC 4 x output index, a pair's fields
        4 x index (top) and 4 x index + 1 (bottom).  B pictures (non-reference unless
        c.b_ref) predict from the reference fields of both lists (8.2.4.2.4); keep direct
        prediction spatial (c.direct = (1,)) -- temporal direct needs the co-located field's
        reference in list 0."""
        c, r = self.c, self.rng
        order, k = [(0, None)], 0
        while k + 1 < c.frames:
            anchor = min(k + c.bframes + 1, c.frames - 1)
            order.append((anchor, None))
            order += [(b, "B") for b in range(k + 1, anchor)]
            k = anchor
        out = []
        for i, (disp, kind) in enumerate(order):
            ref_idc = 3 if kind != "B" else (2 if r.random() < c.b_ref else 0)
            idr = i == 0
            fld = c.field >= 1.0 or r.random() < c.field
            if not fld:
                out += self.picture(i, idr=idr, kind=kind, ref_idc=ref_idc, poc=4 * disp)
                continue
            first = 2 if c.bottom_first and r.random() < c.bottom_first else 1
            ptype = "B" if kind == "B" else ("I" if idr else "P")
            nfr = self.st + self.lt                          # reference frames before this one
            f1 = 2 * nfr
            n1 = (f1, min(f1, 2 * c.l1_refs)) if ptype == "B" else min(f1, H264R_MAX_FIELD_REFS)
            out += self.picture(i, idr=idr, kind=kind, ref_idc=ref_idc, poc=4 * disp + (first == 2),
                                structure=first, nref_field=n1)
            # the second field: the first one is a reference field of the same frame when it is
            # one (the sliding window has counted its frame)
            f2 = 2 * (self.st + self.lt - 1) + 1 if ref_idc else 2 * nfr
            n2 = (f2, min(f2, 2 * c.l1_refs)) if ptype == "B" else min(f2, H264R_MAX_FIELD_REFS)
            out += self.picture(i, idr=False, kind="B" if ptype == "B" else "P", ref_idc=ref_idc,
                                poc=4 * disp + (first == 1), structure=3 - first, second=True, nref_field=n2)
        return out


H264R_MAX_FIELD_REFS = 16                  # the reconstruction ABI's list length (include/h264r.h)


class _Deferred:
    """Writes mb_skip_run (ue) just before the first syntax element of a coded MB in a P
    slice; a skipped MB writes nothing."""

    def __init__(self, w: BitWriter, run: int):
        self.w, self.run, self.done = w, run, False

    def _flush(self):
        if not self.done:
            self.w.ue(self.run)
            self.done = True

    def __getattr__(self, name):
        self._flush()
        return getattr(self.w, name)


def write_stream(path: str, cfg: StreamCfg) -> bytes:
    data = Encoder(cfg).stream()
    with open(path, "wb") as f:
        f.write(data)
    return data
