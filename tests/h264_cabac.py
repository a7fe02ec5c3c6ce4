"""h264_cabac -- the CABAC side of the repo's bitstream writer (TEST INFRASTRUCTURE).

The arithmetic encoder of H.264 9.3.4 (EncodeDecision / EncodeBypass / EncodeTerminate /
EncodeFlush with PutBit's outstanding-bit handling) and the binarisation + context
selection of every syntax element the writer emits, each written as the inverse of the
reference decoder's own reading procedure so that the reference parses back exactly the
decisions the writer made:

    mb_skip_flag, mb_type (I / P / B prefixes and the I suffix)    interpret_se.cc:66-235
    sub_mb_type (P / B)                                            interpret_se.cc:237-292
    transform_size_8x8_flag, prev/rem intra pred mode, intra_chroma_pred_mode,
    ref_idx_lX, mvd_lX, coded_block_pattern, mb_qp_delta           interpret_se.cc:294-456
    ctxIdxInc of each from the neighbouring MBs / blocks            neighbour.cc:415-764
    residual_block_cabac (coded_block_flag, significance map,
    coeff_abs_level_minus1, sign)                                  interpret_residual.cc:272-404
    end_of_slice_flag, I_PCM re-initialisation                     slice_data.cc:526-560, interpret_mb.cc:406-475

The context variables use the reference's own layout (cabac_contexts_t,
bitstream_cabac.h:61-83); their initial values, the engine's state tables and the
residual context maps come from tests/golden/cabac_tables.json, probed from the compiled
reference (oracle/probe_cabac.cc).
"""
from __future__ import annotations

import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
_T = json.load(open(os.path.join(HERE, "golden", "cabac_tables.json")))
FIELD = {name: first for name, first, _count in _T["fields"]}
RANGE_LPS = _T["rangeTabLPS"]
TRANS_LPS = _T["transIdxLPS"]
TRANS_MPS = _T["transIdxMPS"]
POS_MAP = {"4x4": _T["pos2ctx_map4x4"], "8x8": _T["pos2ctx_map8x8"], "2x4c": _T["pos2ctx_map2x4c"]}
# field pictures (shr.field_pic_flag): the significance maps of the second context sets
# map_contexts[1] / last_contexts[1] and, for 8x8 blocks, the field position map
# (interpret_residual.cc:353-358; bitstream_cabac.h:78-79)
POS_MAP_FIELD = dict(POS_MAP, **{"8x8": _T["pos2ctx_map8x8_field"]})
_NFIELD = {name: count for name, _first, count in _T["fields"]}
MAP_SET, LAST_SET = _NFIELD["map_contexts"] // 2, _NFIELD["last_contexts"] // 2
POS_LAST = {"4x4": _T["pos2ctx_last4x4"], "8x8": _T["pos2ctx_last8x8"], "2x4c": _T["pos2ctx_last2x4c"]}
T2C_BCBP, T2C_MAP, T2C_ONE = _T["type2ctx_bcbp"], _T["type2ctx_map"], _T["type2ctx_one"]

# residual block types of residual_block_cabac (interpret_residual.cc:250-265)
LUMA_16DC, LUMA_16AC, LUMA_4x4, CHROMA_DC, CHROMA_AC, LUMA_8x8 = 0, 1, 2, 3, 4, 5
_POS = {LUMA_16DC: "4x4", LUMA_16AC: "4x4", LUMA_4x4: "4x4", CHROMA_DC: "4x4", CHROMA_AC: "4x4", LUMA_8x8: "8x8"}   # (2x4c: 4:2:2 chroma DC)


class CabacEncoder:
    """9.3.4: codILow / codIRange, PutBit with bitsOutstanding, the first bit suppressed."""

    def __init__(self, bits: list):
        self.bits = bits
        self.ctx = None
        self.reset()

    def reset(self) -> None:
        self.low, self.range, self.outstanding, self.first = 0, 510, 0, True

    def init_contexts(self, key: str, qp: int) -> None:
        """9.3.1.1 with the probed (m, n) of slice kind `key` ("I", "P0".."P2", "B0".."B2")."""
        qp = max(0, min(51, qp))
        self.ctx = []
        for mn in _T["init"][key]:
            if mn is None:
                self.ctx.append(None)
                continue
            pre = max(1, min(126, ((mn[0] * qp) >> 4) + mn[1]))
            self.ctx.append([63 - pre, 0] if pre <= 63 else [pre - 64, 1])

    def _put(self, b: int) -> None:
        if self.first:
            self.first = False
        else:
            self.bits.append(b)
        while self.outstanding:
            self.bits.append(1 - b)
            self.outstanding -= 1

    def _renorm(self) -> None:
        while self.range < 256:
            if self.low < 256:
                self._put(0)
            elif self.low >= 512:
                self.low -= 512
                self._put(1)
            else:
                self.low -= 256
                self.outstanding += 1
            self.range <<= 1
            self.low <<= 1

    def decision(self, idx: int, b: int) -> None:
        st = self.ctx[idx]
        lps = RANGE_LPS[st[0]][(self.range >> 6) & 3]
        self.range -= lps
        if b != st[1]:
            self.low += self.range
            self.range = lps
            if st[0] == 0:
                st[1] = 1 - st[1]
            st[0] = TRANS_LPS[st[0]]
        else:
            st[0] = TRANS_MPS[st[0]]
        self._renorm()

    def bypass(self, b: int) -> None:
        self.low <<= 1
        if b:
            self.low += self.range
        if self.low >= 1024:
            self._put(1)
            self.low -= 1024
        elif self.low < 512:
            self._put(0)
        else:
            self.low -= 512
            self.outstanding += 1

    def terminate(self, b: int) -> None:
        self.range -= 2
        if b:
            self.low += self.range
            self.flush()
        else:
            self._renorm()

    def flush(self) -> None:
        """EncodeFlush: the last bit written is 1 (rbsp_stop_one_bit at a slice end)."""
        self.range = 2
        self._renorm()
        self._put((self.low >> 9) & 1)
        v = ((self.low >> 7) & 3) | 1
        self.bits.append(v >> 1)
        self.bits.append(v & 1)


class CabacSink:
    """The writer's syntax elements as CABAC bins (see the module docstring).  `enc` is the
    h264_writer.Encoder (its MB array holds the state the context selection reads)."""

    def __init__(self, enc, bits: list, ptype: str, qp: int, init_idc: int, s: int, field: bool = False):
        self.e = enc
        self.field = field
        self.ptype = ptype
        self.s = s
        self.a = 0
        self.cab = CabacEncoder(bits)
        self.cab.init_contexts("I" if ptype == "I" else f"{ptype}{init_idc}", qp)
        self.last_dquant = 0
        self.log = getattr(enc, "se_log", None)   # debugging: the syntax elements as oracle/_ref/ldecod_trace prints them

    def _log(self, text: str) -> None:
        if self.log is not None:
            self.log.append(text)

    # ---------------------------------------------------------------- neighbours
    def _mb(self, dx: int, dy: int):
        """The MB at (x + dx, y + dy) of the current MB if it is in the current slice (MBAFF: the
        MB holding sample (-1, 0) / (0, -1), get_mb neighbour.cc:175-227)."""
        if self.e.c.mbaff:
            nb = self.e._nbr(self.a, -1 if dx < 0 else 0, -1 if dy < 0 else 0)
            return None if nb is None else nb[0]
        W = self.e.W
        x, y = self.a % W + dx, self.a // W + dy
        return self.e._mb_at(x, y, self.s)

    def _blk(self, bx: int, by: int):
        """(MB, bx & 3, by & 3) of luma 4x4 block (bx, by) relative to the current MB, or None
        (MBAFF: the block holding that block's top-left sample, get_neighbour)."""
        if self.e.c.mbaff and (bx < 0 or by < 0):
            nb = self.e._nbr(self.a, -1 if bx < 0 else bx * 4, -1 if by < 0 else by * 4)   # (x-1, y) / (x, y-1)
            return None if nb is None else (nb[0], nb[1] // 4, nb[2] // 4)
        m = self._mb(-1 if bx < 0 else 0, -1 if by < 0 else 0) if (bx < 0 or by < 0) else self.e.mbs[self.a]
        return None if m is None else (m, bx & 3, by & 3)

    def _dec(self, field: str, inc: int, b: int) -> None:
        self.cab.decision(FIELD[field] + inc, b)

    # ---------------------------------------------------------------- MB header
    def start_mb(self, a: int) -> None:
        self.a = a

    def skip_flag(self, skip: bool) -> None:
        """mb_skip_flag (neighbour.cc:415-427): ctxIdxInc = A, B available and not skipped."""
        inc = sum(1 for m in (self._mb(-1, 0), self._mb(0, -1)) if m is not None and not m.skip)
        self._log(f"mb_skip_flag = {int(skip)}")
        self._dec("skip_contexts", inc, 1 if skip else 0)
        if skip:
            self.last_dquant = 0

    def field_flag(self, fld: bool) -> None:
        """mb_field_decoding_flag (neighbour.cc:429-445): ctxIdxInc = the pairs to the left and
        above in the slice that are field pairs."""
        W = self.e.W
        mx, py = self.a % W, (self.a // W) // 2
        A = self.e.mbs[2 * py * W + mx - 1] if mx > 0 else None
        B = self.e.mbs[(2 * py - 1) * W + mx] if py > 0 else None
        inc = sum(1 for n in (A, B) if n is not None and n.slice == self.s and n.fld)
        self._dec("mb_aff_contexts", inc, 1 if fld else 0)

    def end_of_slice(self, last: bool) -> None:
        self.cab.terminate(1 if last else 0)

    def _i_suffix(self, base: int, v: int, first_inc: int) -> None:
        """I mb_type bins after the prefix: bin 0 at mb_type_contexts[base + first_inc] (I_NxN 0),
        terminate (I_PCM 1), then CBP luma, chroma (two bins) and the 16x16 mode (two bins)
        (interpret_se.cc:123-138; P / B suffixes :160-170 / :210-222 use other offsets)."""
        i_slice = self.ptype == "I"
        o = (lambda k: base + k) if i_slice else (lambda k: base + (0, 1, 2, 2, 3, 3)[k])
        self._dec("mb_type_contexts", base + first_inc if i_slice else base, 0 if v == 0 else 1)
        if v == 0:
            return
        self.cab.terminate(1 if v == 25 else 0)
        if v == 25:
            return
        t = v - 1
        cbpl, cbpc, mode = t // 12, (t % 12) // 4, t % 4
        self._dec("mb_type_contexts", o(3) if i_slice else o(1), cbpl)
        self._dec("mb_type_contexts", o(4) if i_slice else o(2), 1 if cbpc else 0)
        if cbpc:
            self._dec("mb_type_contexts", o(5) if i_slice else o(3), 1 if cbpc == 2 else 0)
        self._dec("mb_type_contexts", o(6) if i_slice else o(4), mode >> 1)
        self._dec("mb_type_contexts", o(7) if i_slice else o(5), mode & 1)

    def mb_type_intra(self, v: int) -> None:
        """mb_type of an intra MB (I-slice numbering: 0 I_NxN, 1..24 I_16x16, 25 I_PCM)."""
        self._log(f"mb_type = {v + {'I': 0, 'P': 5, 'B': 23}[self.ptype]}")
        if self.ptype == "I":
            inc = sum(1 for m in (self._mb(-1, 0), self._mb(0, -1)) if m is not None and m.mbt_ref not in (8, 9))
            self._i_suffix(3, v, inc)
        elif self.ptype == "P":
            self._dec("mb_type_contexts", 0, 1)               # prefix: intra
            self._i_suffix(3, v, 0)
        else:
            self._b_type_bins(23)
            self._i_suffix(5, v, 0)

    def mb_type_p(self, mbt: int) -> None:
        """P mb_type 0..3 (interpret_se.cc:142-157): 0 = 000, 1 = 011, 2 = 010, 3 = 001."""
        self._log(f"mb_type = {mbt}")
        self._dec("mb_type_contexts", 0, 0)
        if mbt in (0, 3):
            self._dec("mb_type_contexts", 1, 0)
            self._dec("mb_type_contexts", 2, 1 if mbt == 3 else 0)
        else:
            self._dec("mb_type_contexts", 1, 1)
            self._dec("mb_type_contexts", 3, 1 if mbt == 1 else 0)

    def _b_type_bins(self, v: int) -> None:
        """B mb_type prefix (interpret_se.cc:176-208); v = 23 is the intra prefix."""
        inc = sum(1 for m in (self._mb(-1, 0), self._mb(0, -1)) if m is not None and m.mbt_ref != 0)
        d = lambda k, b: self._dec("mb_type_contexts", k, b)
        if v == 0:
            d(inc, 0)
            return
        d(inc, 1)
        if v in (1, 2):
            d(3, 0); d(5, v - 1)
            return
        d(3, 1)
        if 3 <= v <= 10:
            d(4, 0)
            t = v - 3
            d(5, t >> 2); d(5, (t >> 1) & 1); d(5, t & 1)
            return
        d(4, 1)
        if v == 11:
            bits = (1, 1, 0)
        elif v == 22:
            bits = (1, 1, 1)
        elif v == 23:
            bits = (1, 0, 1)
        else:
            t = v - 12
            bits = (0, (t >> 2) & 1, (t >> 1) & 1, t & 1) if t < 8 else (1, 0, 0, t - 8)
        for b in bits:
            d(5, b)

    def mb_type_b(self, mbt: int) -> None:
        self._log(f"mb_type = {mbt}")
        self._b_type_bins(mbt)

    def sub_p(self, sb: int) -> None:
        """P sub_mb_type (interpret_se.cc:252-264): 0 = 1, 1 = 00, 2 = 011, 3 = 010."""
        self._log(f"sub_mb_type = {sb}")
        d = lambda k, b: self._dec("b8_type_contexts", k, b)
        if sb == 0:
            d(0, 1)
            return
        d(0, 0)
        if sb == 1:
            d(1, 0)
        else:
            d(1, 1); d(2, 1 if sb == 2 else 0)

    def sub_b(self, sb: int) -> None:
        """B sub_mb_type (interpret_se.cc:266-289)."""
        self._log(f"sub_mb_type = {sb}")
        d = lambda k, b: self._dec("b8_type_contexts", k, b)
        if sb == 0:
            d(0, 0)
            return
        d(0, 1)
        if sb <= 2:
            d(1, 0); d(3, sb - 1)
            return
        d(1, 1)
        if sb <= 6:
            d(2, 0); d(3, (sb - 3) >> 1); d(3, (sb - 3) & 1)
        elif sb <= 10:
            d(2, 1); d(3, 0); d(3, (sb - 7) >> 1); d(3, (sb - 7) & 1)
        else:
            d(2, 1); d(3, 1); d(3, sb - 11)

    def transform8x8(self, flag: bool) -> None:
        self._log(f"transform_size_8x8_flag = {int(flag)}")
        inc = sum(1 for m in (self._mb(-1, 0), self._mb(0, -1)) if m is not None and m.t8)
        self._dec("transform_size_contexts", inc, 1 if flag else 0)

    def intra_mode(self, mode: int, pred: int) -> None:
        """prev flag at ipr_contexts[0]; rem as 3 bins, LSB first, at ipr_contexts[1] (fl)."""
        self._log(f"intra_pred_mode = {-1 if mode == pred else (mode if mode < pred else mode - 1)}")
        if mode == pred:
            self._dec("ipr_contexts", 0, 1)
            return
        self._dec("ipr_contexts", 0, 0)
        rem = mode if mode < pred else mode - 1
        for k in range(3):
            self._dec("ipr_contexts", 1, (rem >> k) & 1)

    def chroma_mode(self, v: int) -> None:
        """TU, cMax 3; bin 0 at inc (A / B intra with a non-DC chroma mode), bins 1.. at 3."""
        self._log(f"intra_chroma_pred_mode = {v}")
        inc = sum(1 for m in (self._mb(-1, 0), self._mb(0, -1))
                  if m is not None and m.cmode != 0 and m.mbt_ref != 12)
        for k in range(v):
            self._dec("cipr_contexts", inc if k == 0 else 3, 1)
        if v < 3:
            self._dec("cipr_contexts", inc if v == 0 else 3, 0)

    def cbp(self, cbp: int) -> None:
        """coded_block_pattern (interpret_se.cc:424-442, neighbour.cc:645-699)."""
        self._log(f"coded_block_pattern = {cbp}")
        cur = 0
        for b8 in range(4):
            x0, y0 = (b8 & 1) * 2, (b8 >> 1) * 2
            if x0 == 0:
                nb = self._blk(-1, y0)                     # the left 8x8 block of this row (MBAFF: its row)
                m = None if nb is None else nb[0]
                ca, ia = (m.cbpl, (nb[2] & ~1) + 1) if (m is not None and m.mbt_ref != 12) else (0x3F, 0)
            else:
                ca, ia = cur, y0
            if y0 == 0:
                m = self._mb(0, -1)
                cb, ib = (m.cbpl, x0 // 2 + 2) if (m is not None and m.mbt_ref != 12) else (0x3F, 0)
            else:
                cb, ib = cur, x0 // 2
            inc = (0 if ca & (1 << ia) else 1) + 2 * (0 if cb & (1 << ib) else 1)
            bit = (cbp >> b8) & 1
            self._dec("cbp_l_contexts", inc, bit)
            cur |= bit << (y0 + (x0 >> 1))
        A, B = self._mb(-1, 0), self._mb(0, -1)
        f = lambda m, two: m is not None and (m.mbt_ref == 12 or (m.cbpc == 2 if two else m.cbpc != 0))
        cbpc = cbp >> 4
        if self.e.c.chroma_format in (0, 3):          # no chroma bins (interpret_se.cc:429)
            if not cbp:
                self.last_dquant = 0
            return
        self._dec("cbp_c_contexts", int(f(A, False)) + 2 * int(f(B, False)), 1 if cbpc else 0)
        if cbpc:
            self._dec("cbp_c_contexts", int(f(A, True)) + 2 * int(f(B, True)) + 4, 1 if cbpc == 2 else 0)
        if not cbp:
            self.last_dquant = 0

    def qp_delta(self, d: int) -> None:
        """mb_qp_delta: unary of 2|d| - (d > 0) at delta_qp_contexts {last != 0, 2, 3}."""
        self._log(f"mb_qp_delta = {d}")
        n = 2 * d - 1 if d > 0 else -2 * d
        first = 1 if self.last_dquant != 0 else 0
        for k in range(n):
            self._dec("delta_qp_contexts", first if k == 0 else (2 if k == 1 else 3), 1)
        self._dec("delta_qp_contexts", first if n == 0 else (2 if n == 1 else 3), 0)
        self.last_dquant = d

    def _ueg(self, field: str, incs: list, cmax: int, k: int, v: int, signed: bool) -> None:
        """UEGk with a TU prefix (cMax) and bypass suffix (interpret.cc:402-422)."""
        a = abs(v)
        pre = min(a, cmax)
        for i in range(pre):
            self._dec(field, incs[min(i, len(incs) - 1)], 1)
        if a < cmax:
            self._dec(field, incs[min(a, len(incs) - 1)], 0)
        else:
            s = a - cmax
            while s >= (1 << k):
                self.cab.bypass(1)
                s -= 1 << k
                k += 1
            self.cab.bypass(0)
            while k:
                k -= 1
                self.cab.bypass((s >> k) & 1)
        if signed and a:
            self.cab.bypass(1 if v < 0 else 0)

    def _part_neighbours(self, x0: int, y0: int):
        """Neighbours A (x0-1, y0) and B (x0, y0-1) of a partition's top-left 4x4 block."""
        return self._blk(x0 - 1, y0), self._blk(x0, y0 - 1)

    def _coded_part(self, nb) -> bool:
        """A neighbour partition with coded motion: not skipped / direct / intra, and its
        SubMbType non-zero (neighbour.cc:520-566: predModeEqualFlag)."""
        m, bx, by = nb
        if m.skip or m.intra or m.mbt_ref == 0:
            return False
        return not m.sub_direct[(by >> 1) * 2 + (bx >> 1)]

    def ref_idx(self, v: int, n: int, lst: int, x0: int, y0: int) -> None:
        self._log(f"ref_idx {lst} {x0} {y0} = {v}")          # (the parser's reader is called either way)
        if n <= 1:
            return
        inc = 0
        for w, nb in zip((1, 2), self._part_neighbours(x0, y0)):
            if nb is not None and self._coded_part(nb):
                m, bx, by = nb
                # a frame MB over a field neighbour: refIdx > 1 (neighbour.cc:533-536)
                lim = 1 if (self.e.c.mbaff and not self.e.mbs[self.a].fld and m.fld) else 0
                if m.ref[lst][by * 4 + bx] > lim:
                    inc += w
        incs = [inc, 4, 5]
        for k in range(v):
            self._dec("ref_no_contexts", incs[min(k, 2)], 1)
        self._dec("ref_no_contexts", incs[min(v, 2)], 0)

    def mvd(self, v: int, lst: int, comp: int, x0: int, y0: int) -> None:
        self._log(f"mvd {lst} {x0} {y0} {comp} = {v}")
        s = 0
        for nb in self._part_neighbours(x0, y0):
            if nb is not None and self._coded_part(nb):
                m, bx, by = nb
                av = abs(m.mvd[lst][by * 4 + bx][comp])
                if self.e.c.mbaff and comp:                # field / frame units (neighbour.cc:599-604)
                    cf = self.e.mbs[self.a].fld
                    av = av * 2 if (not cf and m.fld) else (av // 2 if (cf and not m.fld) else av)
                s += av
        inc = 0 if s < 3 else (1 if s <= 32 else 2)
        self._ueg("mvd_x_contexts" if comp == 0 else "mvd_y_contexts", [inc, 3, 4, 5, 6], 9, 3, v, True)

    # ---------------------------------------------------------------- residual
    def _cbf_inc(self, typ: int, pl: int, blk: int) -> int:
        """coded_block_flag ctxIdxInc (neighbour.cc:689-740) from the neighbours' cbp_bits."""
        m_cur = self.e.mbs[self.a]
        chroma = typ in (CHROMA_DC, CHROMA_AC)
        ac = typ not in (LUMA_16DC, CHROMA_DC)
        if chroma:
            i, j = blk % 2, blk // 2
        else:
            i, j = ((blk // 4) % 2) * 2 + (blk % 4) % 2, ((blk // 4) // 2) * 2 + (blk % 4) // 2
        if not chroma:
            bit = 0 if not ac else 1
        else:
            bit = (17 if pl == 1 else 18) if not ac else (19 if pl == 1 else 35)
        inc = 0
        for w, (di, dj) in ((1, (-1, 0)), (2, (0, -1))):
            ni, nj = i + di, j + dj
            if ni >= 0 and nj >= 0:
                m, pi, pj = m_cur, ni, nj
            elif self.e.c.mbaff:                            # get_neighbour of the block's sample
                nb = self.e._nbr(self.a, -1 if ni < 0 else ni * 4, -1 if nj < 0 else nj * 4, chroma)
                if nb is None:
                    inc += w if m_cur.intra else 0
                    continue
                m, pi, pj = nb[0], nb[1] // 4, nb[2] // 4
            else:
                m = self._mb(-1 if ni < 0 else 0, -1 if nj < 0 else 0)
                if m is None:
                    inc += w if m_cur.intra else 0
                    continue
                nw = 2 if chroma else 4                     # 4x4 blocks per MB: 4:2:2 chroma 2 x 4
                nh = (4 if self.e.c.chroma_format == 2 else 2) if chroma else 4
                pi, pj = ni % nw, nj % nh
            if m.mbt_ref == 12:
                inc += w
                continue
            pos = (pj * 4 + pi) if ac else 0
            inc += w * ((m.cbp_bits >> (bit + pos)) & 1)
        return inc

    def block(self, typ: int, pl: int, blk: int, coeffs: list) -> None:
        """residual_block_cabac of `coeffs` (the block's coefficients in scan order, from its
        start index) of type `typ`, plane pl, block index blk."""
        m_cur = self.e.mbs[self.a]
        coded = any(coeffs)
        if typ != LUMA_8x8:
            self._dec("bcbp_contexts", T2C_BCBP[typ] + self._cbf_inc(typ, pl, blk), 1 if coded else 0)
        if not coded:
            return
        # update_coded_block_flag (neighbour.cc:742-764)
        chroma = typ in (CHROMA_DC, CHROMA_AC)
        ac = typ not in (LUMA_16DC, CHROMA_DC)
        if chroma:
            i, j = blk % 2, blk // 2
        else:
            i, j = ((blk // 4) % 2) * 2 + (blk % 4) % 2, ((blk // 4) // 2) * 2 + (blk % 4) // 2
        bit = (0 if not ac else 1) if not chroma else ((17 if pl == 1 else 18) if not ac else (19 if pl == 1 else 35))
        m_cur.cbp_bits |= (0x33 if typ == LUMA_8x8 else 0x01) << (bit + (j * 4 + i if ac else 0))
        n = len(coeffs)
        last = max(k for k, v in enumerate(coeffs) if v)
        pos = "2x4c" if typ == CHROMA_DC and self.e.c.chroma_format == 2 else _POS[typ]   # CHROMA_DC_2x4 maps
        fld = self.field or m_cur.fld                      # field pictures and field MBs
        pm, pl_ = (POS_MAP_FIELD if fld else POS_MAP)[pos], POS_LAST[pos]
        fm, fl = (MAP_SET, LAST_SET) if fld else (0, 0)
        for k in range(n - 1):
            sig = 1 if coeffs[k] else 0
            self._dec("map_contexts", fm + T2C_MAP[typ] + pm[k], sig)
            if sig:
                self._dec("last_contexts", fl + T2C_MAP[typ] + pl_[k], 1 if k == last else 0)
                if k == last:
                    break
        eq1 = gt1 = 0
        for k in range(last, -1, -1):
            v = coeffs[k]
            if not v:
                continue
            am1 = abs(v) - 1
            inc0 = 0 if gt1 else min(4, 1 + eq1)
            inc1 = 5 + min(4 - (1 if typ == CHROMA_DC else 0), gt1)
            one = T2C_ONE[typ]
            self._dec("one_contexts", one + inc0, 1 if am1 else 0)
            if am1:
                pre = min(am1 - 1, 13)
                for _ in range(pre):
                    self._dec("one_contexts", one + inc1, 1)
                if am1 - 1 < 13:
                    self._dec("one_contexts", one + inc1, 0)
                else:
                    s, kk = am1 - 14, 0
                    while s >= (1 << kk):
                        self.cab.bypass(1)
                        s -= 1 << kk
                        kk += 1
                    self.cab.bypass(0)
                    while kk:
                        kk -= 1
                        self.cab.bypass((s >> kk) & 1)
            self.cab.bypass(1 if v < 0 else 0)
            start = 1 if typ in (LUMA_16AC, CHROMA_AC) else 0
            name = ("coeff_chroma_" if chroma else "coeff_luma_") + ("ac" if ac else "dc")
            self._log(f"{name} {pl} {i} {j} {k + start} = {v}")
            eq1 += am1 == 0
            gt1 += am1 != 0

    def pcm(self, samples: list) -> None:
        """After mb_type I_PCM (terminate 1 + flush): pcm_alignment_zero_bits, the samples,
        then the engine restarts (contexts kept)."""
        bits = self.cab.bits
        while len(bits) % 8:
            bits.append(0)
        for v in samples:
            for k in range(7, -1, -1):
                bits.append((v >> k) & 1)
        self.cab.reset()
        self.last_dquant = 0
