// mb_deblock2.h -- packed 16-bit deblocking filters on register-resident lines, gfx950.
//
// filter_edge / filter_normal / filter_strong (deblock.cc:327-486) evaluated on two lines
// at once: every operand is an s16x2 {line a, line b} of samples 0..255, and every
// decision (filterSamplesFlag, ap < beta, aq < beta, the strong-filter condition, bS == 4,
// bS == 0) is a 16-bit sign mask (0 or -1 per half) built with subtract + arithmetic
// shift, so no per-half compare or branch is needed (v_pk_* VALU, one instruction per two
// lines).  The two halves may carry different bS (and tc0); alpha / beta are the edge's.
#pragma once
#include "device_common.h"

namespace h264r {

typedef short s2 __attribute__((ext_vector_type(2)));
typedef unsigned short u2 __attribute__((ext_vector_type(2)));

DEV s2 sp2(short v) { return (s2){v, v}; }
DEV s2 as_s2(uint32_t v) { return __builtin_bit_cast(s2, v); }
DEV uint32_t as_w(s2 v) { return __builtin_bit_cast(uint32_t, v); }
DEV s2 smin(s2 a, s2 b) { return __builtin_elementwise_min(a, b); }
DEV s2 smax(s2 a, s2 b) { return __builtin_elementwise_max(a, b); }
DEV s2 absd(s2 a, s2 b)                        // |a - b| of samples 0..255
{
    const u2 ua = __builtin_bit_cast(u2, a), ub = __builtin_bit_cast(u2, b);
    return __builtin_bit_cast(s2, (u2)(__builtin_elementwise_max(ua, ub) - __builtin_elementwise_min(ua, ub)));
}
DEV s2 neg_mask(s2 v) { return v >> sp2(15); }  // -1 where v < 0, else 0
DEV s2 sel(s2 m, s2 a, s2 b)                    // m (-1 / 0 per half) ? a : b
{
    return as_s2((as_w(m) & as_w(a)) | (~as_w(m) & as_w(b)));
}
DEV s2 clamp255(s2 v) { return smin(smax(v, sp2(0)), sp2(255)); }
// A mask the compiler must not look through: seen as a sign splat, it became per-half lane
// compares and every sel() on it two selects plus a re-pack instead of one bitfield insert.
DEV s2 opaque_mask(s2 m)
{
    uint32_t w = as_w(m);
    asm volatile("" : "+v"(w));
    return as_s2(w);
}

// {byte b of A, byte b of B} as an s16x2 (A in the low half).
DEV s2 unpack2(uint32_t A, uint32_t B, int b)
{
    return as_s2(__builtin_amdgcn_perm(B, A, 0x0C000C00u | ((uint32_t)(4 + b) << 16) | (uint32_t)b));
}
// The low / high halves of four s16x2 (columns 0..3) as two dwords of bytes.
DEV void pack4(s2 c0, s2 c1, s2 c2, s2 c3, uint32_t& lo, uint32_t& hi)
{
    const uint32_t u = __builtin_amdgcn_perm(as_w(c1), as_w(c0), 0x06020400u);   // {lo0, lo1, hi0, hi1}
    const uint32_t v = __builtin_amdgcn_perm(as_w(c3), as_w(c2), 0x06020400u);   // {lo2, lo3, hi2, hi3}
    lo = __builtin_amdgcn_perm(v, u, 0x05040100u);
    hi = __builtin_amdgcn_perm(v, u, 0x07060302u);
}

// Bytes 2*half, 2*half+1 of lo / hi replaced by the low / high halves of c0, c1.
DEV void merge2(s2 c0, s2 c1, int half, uint32_t& lo, uint32_t& hi)
{
    const uint32_t u = __builtin_amdgcn_perm(as_w(c1), as_w(c0), 0x06020400u);   // {lo0, lo1, hi0, hi1}
    // perm selectors: 0..3 = bytes of the second operand (u), 4..7 = the first (lo / hi)
    lo = __builtin_amdgcn_perm(lo, u, half ? 0x01000504u : 0x07060100u);
    hi = __builtin_amdgcn_perm(hi, u, half ? 0x03020504u : 0x07060302u);
}

// Per-edge parameters of the two halves: alpha / beta of the edge, bS and tc0 per half.
struct EdgeP {
    s2 am1, bm1;        // alpha - 1, beta - 1
    s2 bs;              // bS per half
    s2 tc0;             // tc0(bS) per half (0 for bS 0 and 4)
    s2 alpha;
};

// par = edge_word() (mb_deblock.h): alpha | beta << 8 | tc0(bS 1..3) << 16 / 21 / 26.
// bs2 = {bS of half a, bS of half b}.
DEV EdgeP edge_params(uint32_t par, s2 bs2)
{
    EdgeP e;
    const short alpha = (short)(par & 255), beta = (short)((par >> 8) & 255);
    e.alpha = sp2(alpha);
    e.am1 = sp2((short)(alpha - 1));
    e.bm1 = sp2((short)(beta - 1));
    e.bs = bs2;
    // tc0(bS) of each half by one byte permute: bS (0..4, the half's low byte) indexes the
    // bytes {0, tc0(1), tc0(2), tc0(3)} and, for bS 4, byte 0 of a zero operand
    const uint32_t T = (((par >> 16) & 31) << 8) | (((par >> 21) & 31) << 16) | (((par >> 26) & 31) << 24);
    e.tc0 = as_s2(__builtin_amdgcn_perm(0u, T, as_w(bs2) | 0x0c000c00u));
    return e;
}

// filterSamplesFlag and friends for luma (chroma = false) or chroma lines;
// STRONG: some half of the wave may have bS == 4 (MB edges only).
template <bool STRONG, bool CHROMA>
DEV void filter2(s2& p3, s2& p2, s2& p1, s2& p0, s2& q0, s2& q1, s2& q2, s2& q3, const EdgeP& e)
{
    const s2 dpq = absd(p0, q0);
    // -1 where NOT (bS != 0 && |p0-q0| < alpha && |p1-p0| < beta && |q1-q0| < beta)
    const s2 nf = neg_mask(smin(smin(e.am1 - dpq, e.bm1 - absd(p1, p0)), smin(e.bm1 - absd(q1, q0), e.bs - sp2(1))));
    if (CHROMA) {
        // filter_normal, chromaStyleFilteringFlag: tc = tc0 + 1, p0 / q0 only (deblock.cc:380-400)
        const s2 tc = e.tc0 + sp2(1);
        s2 d = ((q0 - p0) * sp2(4) + (p1 - q1) + sp2(4)) >> sp2(3);
        d = smin(smax(d, -tc), tc);
        s2 np0 = clamp255(p0 + d), nq0 = clamp255(q0 - d);
        if (STRONG) {                                  // filter_strong, chroma (deblock.cc:350-364)
            const s2 is4 = opaque_mask(neg_mask(e.bs - sp2(4)) ^ sp2(-1));          // -1 where bS >= 4
            np0 = sel(is4, (p1 * sp2(2) + p0 + q1 + sp2(2)) >> sp2(2), np0);
            nq0 = sel(is4, (q1 * sp2(2) + q0 + p1 + sp2(2)) >> sp2(2), nq0);
        }
        p0 = sel(nf, p0, np0);
        q0 = sel(nf, q0, nq0);
        return;
    }
    const s2 nap = neg_mask(e.bm1 - absd(p2, p0));         // -1 where NOT (|p2-p0| < beta)
    const s2 naq = neg_mask(e.bm1 - absd(q2, q0));
    // filter_normal (deblock.cc:372-415)
    const s2 tc = e.tc0 + sp2(2) + nap + naq;               // tc0 + (ap < beta) + (aq < beta)
    s2 d = ((q0 - p0) * sp2(4) + (p1 - q1) + sp2(4)) >> sp2(3);
    d = smin(smax(d, -tc), tc);
    s2 np0 = clamp255(p0 + d), nq0 = clamp255(q0 - d);
    const s2 avg = (p0 + q0 + sp2(1)) >> sp2(1);
    s2 np1 = sel(nap, p1, p1 + smin(smax((p2 + avg - p1 * sp2(2)) >> sp2(1), -e.tc0), e.tc0));
    s2 nq1 = sel(naq, q1, q1 + smin(smax((q2 + avg - q1 * sp2(2)) >> sp2(1), -e.tc0), e.tc0));
    s2 np2 = p2, nq2 = q2;
    if (STRONG) {                                          // filter_strong (deblock.cc:327-370)
        const s2 is4 = opaque_mask(neg_mask(e.bs - sp2(4)) ^ sp2(-1));
        const s2 nstrong = neg_mask(((e.alpha >> sp2(2)) + sp2(1)) - dpq);   // NOT (|p0-q0| < (alpha >> 2) + 2)
        const s2 nsp = nap | nstrong, nsq = naq | nstrong;
        const s2 s_p0 = sel(nsp, (p1 * sp2(2) + p0 + q1 + sp2(2)) >> sp2(2),
                            (p2 + p1 * sp2(2) + p0 * sp2(2) + q0 * sp2(2) + q1 + sp2(4)) >> sp2(3));
        const s2 s_p1 = sel(nsp, p1, (p2 + p1 + p0 + q0 + sp2(2)) >> sp2(2));
        const s2 s_p2 = sel(nsp, p2, (p3 * sp2(2) + p2 * sp2(3) + p1 + p0 + q0 + sp2(4)) >> sp2(3));
        const s2 s_q0 = sel(nsq, (q1 * sp2(2) + q0 + p1 + sp2(2)) >> sp2(2),
                            (p1 + p0 * sp2(2) + q0 * sp2(2) + q1 * sp2(2) + q2 + sp2(4)) >> sp2(3));
        const s2 s_q1 = sel(nsq, q1, (p0 + q0 + q1 + q2 + sp2(2)) >> sp2(2));
        const s2 s_q2 = sel(nsq, q2, (q3 * sp2(2) + q2 * sp2(3) + q1 + q0 + p0 + sp2(4)) >> sp2(3));
        np0 = sel(is4, s_p0, np0); nq0 = sel(is4, s_q0, nq0);
        np1 = sel(is4, s_p1, np1); nq1 = sel(is4, s_q1, nq1);
        np2 = sel(is4, s_p2, p2);  nq2 = sel(is4, s_q2, q2);
        p2 = sel(nf, p2, np2);
        q2 = sel(nf, q2, nq2);
    }
    p1 = sel(nf, p1, np1);
    p0 = sel(nf, p0, np0);
    q0 = sel(nf, q0, nq0);
    q1 = sel(nf, q1, nq1);
}

}  // namespace h264r
