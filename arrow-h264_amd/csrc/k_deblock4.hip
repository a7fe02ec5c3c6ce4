// k_deblock4.hip -- the in-loop deblocking filter, FOUR MB rows per wave, packed
// 16-bit arithmetic (two sample lines per lane).
//
// Reference: Deblock::deblock_pic deblock.cc:537-552 (raster order, vertical edges
// then horizontal edges per MB), filter_edge :418-485, filter_strong /
// filter_normal :327-415, Tables 8-16/8-17 :294-324.  The order dependence: MB
// (x,y)'s top edge reads samples that MB (x+1,y-1)'s left edge wrote, so MB (x,y)
// may start once (x+1,y-1) is done -- a wavefront with a 2-MB lag per row.
//
// Work unit: one 64-lane wave owns four consecutive MB rows ("quarters", 16 lanes
// each) of one picture; quarter q walks its row two MBs behind quarter q-1, so each
// step filters four MBs with the same instructions.  In a quarter, lanes 0..7 carry
// two luma lines each and lanes 8..15 two chroma lines each (Cb 8..11, Cr 12..15):
// every edge of a line pair is filtered with packed 16-bit operations (v_pk_*), the
// decisions as per-half masks, so one instruction serves two lines.  Vertical edges
// run along rows, horizontal edges along column pairs of the same LDS tiles.
//
// Hand-offs: quarter q -> q+1 through an LDS ring (bottom four rows of each MB);
// quarter 3 -> the next wave's quarter 0 through a self-validating record per MB in
// global memory (32 naturally aligned 8-byte granules {data, launch epoch}, written
// with write-through sc1 stores, read with sc1 loads and re-polled until every granule
// carries this launch's epoch: MI355X_MICROARCH.md hand-off granules).  Waves take
// (row quad, picture) tickets in quad-major order, so a wave only waits on tickets
// taken earlier by running waves: deadlock-free; every spin is bounded.
//
// Sample ownership: after a step the 16x16 (chroma 8x8) block at rows -3..12 and
// columns -4..11 of the MB is final and is stored once, by this quarter; the right
// four columns are carried into the next step, the bottom three rows are stored by
// the row below (or by the last row itself).
#include "mb_inter4.h"

using namespace h264r;

namespace {

constexpr int QP = 8;                       // tile row pitch (dwords)
constexpr int LROWS = 20;                   // luma tile rows -4..15
constexpr int CROWS = 12;                   // chroma tile rows -4..7
constexpr int LBASE = 3;                    // luma row: [3] left strip, [4..7] MB cols 0..15
constexpr int CB_BASE = 3;                  // chroma row: [3] Cb left, [4..5] Cb MB cols 0..7
constexpr int CR_BASE = 0;                  //             [0] Cr left, [1..2] Cr MB cols 0..7
constexpr int DRING = 4;                    // quarter -> quarter ring depth (lag 2)
constexpr unsigned SPIN_LIMIT = 1u << 22;

struct alignas(16) QuarterLds {
    uint32_t y[LROWS * QP];
    uint32_t c[CROWS * QP];
    uint32_t info[DBINFO_DWORDS];
};

struct alignas(16) WaveLds {
    QuarterLds q[4];
    RingEntry ring[4][DRING];
};

DEV uint64_t ld_cc64(const uint64_t* p)
{
    return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DEV void st_cc64(uint64_t* p, uint64_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// ---- packed decisions: masks are 0xFFFF / 0 per 16-bit half
DEV s16x2 lt_mask(s16x2 a, s16x2 b) { return (a - b) >> splat16(15); }        // a < b (|a|,|b| <= 255)
DEV s16x2 absdiff(s16x2 a, s16x2 b) { return pk_max(a - b, b - a); }
DEV s16x2 sel(s16x2 m, s16x2 a, s16x2 b) { return as_s16x2((as_u32(m) & as_u32(a)) | (~as_u32(m) & as_u32(b))); }
DEV s16x2 pk_clip3(s16x2 lo, s16x2 hi, s16x2 x) { return pk_min(pk_max(x, lo), hi); }

// One edge of two lines (filter_edge deblock.cc:459-485 -> filter_strong / filter_normal
// :327-415), branch-free: P3..Q3 hold (line 0, line 1) pairs of p3..q3; bS and the
// edge word are the same for both lines.  Chroma lines use tc0 + 1 and never change
// p1/q1 or take the strong 3-tap path.
// STRONG = false: no line of the wave has bS 4 on this edge (internal edges never do,
// MB edges only next to an intra MB), so the strong filter is not evaluated at all.
template <bool STRONG>
DEV void filter_edge_pk(s16x2& P3, s16x2& P2, s16x2& P1, s16x2& P0, s16x2& Q0, s16x2& Q1, s16x2& Q2, s16x2& Q3,
                        int bS, uint32_t par, bool chroma)
{
    const short alpha = par & 255, beta = (par >> 8) & 255;
    const short tc0 = (bS >= 1 && bS <= 3) ? (short)((par >> (11 + 5 * bS)) & 31) : 0;
    const s16x2 A = splat16(alpha), Bt = splat16(beta);
    const s16x2 dpq = absdiff(P0, Q0);
    const s16x2 on = splat16(bS != 0 ? (short)-1 : 0);
    const s16x2 filt = on & lt_mask(dpq, A) & lt_mask(absdiff(P1, P0), Bt) & lt_mask(absdiff(Q1, Q0), Bt);
    const s16x2 luma = splat16(chroma ? 0 : (short)-1);
    const s16x2 ap = lt_mask(absdiff(P2, P0), Bt) & luma, aq = lt_mask(absdiff(Q2, Q0), Bt) & luma;
    // bS < 4
    const s16x2 tc = chroma ? splat16((short)(tc0 + 1)) : splat16(tc0) - ap - aq;
    const s16x2 delta = pk_clip3(-tc, tc, (((Q0 - P0) << splat16(2)) + (P1 - Q1) + splat16(4)) >> splat16(3));
    const s16x2 n_p0 = pk_clip255(P0 + delta), n_q0 = pk_clip255(Q0 - delta);
    const s16x2 avg = (P0 + Q0 + splat16(1)) >> splat16(1);
    const s16x2 T0 = splat16(tc0);
    const s16x2 n_p1 = sel(ap, P1 + pk_clip3(-T0, T0, (P2 + avg - (P1 << splat16(1))) >> splat16(1)), P1);
    const s16x2 n_q1 = sel(aq, Q1 + pk_clip3(-T0, T0, (Q2 + avg - (Q1 << splat16(1))) >> splat16(1)), Q1);
    if (!STRONG) {
        P1 = sel(filt, n_p1, P1); P0 = sel(filt, n_p0, P0);
        Q0 = sel(filt, n_q0, Q0); Q1 = sel(filt, n_q1, Q1);
        return;
    }
    // bS == 4
    const s16x2 strong = lt_mask(dpq, splat16((short)((alpha >> 2) + 2)));
    const s16x2 sp = ap & strong, sq = aq & strong;
    const s16x2 s_p0 = sel(sp, (P2 + (P1 << splat16(1)) + (P0 << splat16(1)) + (Q0 << splat16(1)) + Q1 + splat16(4)) >> splat16(3),
                           ((P1 << splat16(1)) + P0 + Q1 + splat16(2)) >> splat16(2));
    const s16x2 s_p1 = sel(sp, (P2 + P1 + P0 + Q0 + splat16(2)) >> splat16(2), P1);
    const s16x2 s_p2 = sel(sp, ((P3 << splat16(1)) + P2 + (P2 << splat16(1)) + P1 + P0 + Q0 + splat16(4)) >> splat16(3), P2);
    const s16x2 s_q0 = sel(sq, (P1 + (P0 << splat16(1)) + (Q0 << splat16(1)) + (Q1 << splat16(1)) + Q2 + splat16(4)) >> splat16(3),
                           ((Q1 << splat16(1)) + Q0 + P1 + splat16(2)) >> splat16(2));
    const s16x2 s_q1 = sel(sq, (P0 + Q0 + Q1 + Q2 + splat16(2)) >> splat16(2), Q1);
    const s16x2 s_q2 = sel(sq, ((Q3 << splat16(1)) + Q2 + (Q2 << splat16(1)) + Q1 + Q0 + P0 + splat16(4)) >> splat16(3), Q2);
    const bool is4 = bS == 4;
    P2 = sel(filt, is4 ? s_p2 : P2, P2);
    P1 = sel(filt, is4 ? s_p1 : n_p1, P1);
    P0 = sel(filt, is4 ? s_p0 : n_p0, P0);
    Q0 = sel(filt, is4 ? s_q0 : n_q0, Q0);
    Q1 = sel(filt, is4 ? s_q1 : n_q1, Q1);
    Q2 = sel(filt, is4 ? s_q2 : Q2, Q2);
}

// (byte c of a, byte c of b) as a pair
template <int C>
DEV s16x2 pair_of(uint32_t a, uint32_t b)
{
    return as_s16x2(__builtin_amdgcn_perm(b, a, 0x0c000c00u | ((4u + C) << 16) | C));
}
// dword of the low (H = 0) or high (H = 1) lines of four pairs
template <int H>
DEV uint32_t dword_of(s16x2 x0, s16x2 x1, s16x2 x2, s16x2 x3)
{
    constexpr uint32_t b = H ? 2 : 0;
    const uint32_t lo = __builtin_amdgcn_perm(as_u32(x1), as_u32(x0), 0x0c0c0000u | ((4 + b) << 8) | b);
    const uint32_t hi = __builtin_amdgcn_perm(as_u32(x3), as_u32(x2), ((4 + b) << 24) | (b << 16) | 0x0c0cu);
    return lo | hi;
}

}  // namespace

// hb: hand-off records [pic][quad][W][32] granules {RingEntry dword, epoch}; sync[0]
// the ticket counter; rows: the MB rows of this launch (a band, h264r_decode_batch_rows).
extern "C" __global__ __launch_bounds__(64) void k_deblock4(h264r_batch b, const DbInfo* __restrict__ dbinfo,
                                                           uint64_t* hb, int* sync, int* err, uint32_t epoch, int2 rows)
{
    __shared__ WaveLds L;
    const int lane = threadIdx.x, qd = lane >> 4, ql = lane & 15;
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int W = g.wmb, R0 = rows.x, R1 = rows.y, nquads = (R1 - R0 + 3) >> 2;

    int tk = 0;
    if (lane == 0) tk = atomicAdd(&sync[0], 1);
    const int ticket = __builtin_amdgcn_readfirstlane(tk);
    const int wq = ticket / b.num_pics, pic = ticket % b.num_pics;
    const int r = R0 + 4 * wq + qd;                            // this quarter's MB row
    const bool row_on = r < R1;
    const bool last_row = r == R1 - 1;
    const int nq_on = min(4, R1 - (R0 + 4 * wq));            // quarters with a row
    const bool feeds_ring = qd + 1 < nq_on;                     // q -> q+1 through LDS
    const bool feeds_hb = qd == nq_on - 1 && wq + 1 < nquads;   // last quarter -> next wave
    const uint64_t* hb_in = wq > 0 ? hb + ((size_t)pic * nquads + wq - 1) * W * 32 : nullptr;
    uint64_t* hb_out = hb + ((size_t)pic * nquads + wq) * W * 32;
    const uint64_t tag = (uint64_t)epoch << 32;
    const int steps = W + 2 * (nq_on - 1);

    QuarterLds& S = L.q[qd];
    uint8_t* Y = b.out_y + (size_t)pic * g.ysz;
    uint8_t* Cp[2] = {b.out_u + (size_t)pic * g.csz, b.out_v + (size_t)pic * g.csz};
    const int Y0 = r * 16, Yc = r * 8;
    const uint32_t* info_row = reinterpret_cast<const uint32_t*>(dbinfo + (size_t)pic * g.nmb + (size_t)min(r, R1 - 1) * W);

    // ---- lane roles
    const bool luma = ql < 8;
    const int cpl = (ql >> 2) & 1;                              // chroma lanes: 8..11 Cb, 12..15 Cr
    const int line0 = luma ? 2 * ql : 2 * (ql & 3);             // first of my two lines / columns
    uint32_t* T = luma ? S.y : S.c;
    const int base = luma ? LBASE : (cpl ? CR_BASE : CB_BASE);  // dword of the left strip in a tile row
    const int seg = luma ? ql >> 1 : ql & 3;                    // bS segment of my lines / columns
    const uint8_t* ib = reinterpret_cast<const uint8_t*>(S.info);
    const int pe = luma ? 8 : 11 + 3 * cpl, pi = luma ? 10 : 13 + 3 * cpl;

    uint4 pf_y = make_uint4(0, 0, 0, 0);
    uint2 pf_c = make_uint2(0, 0), pf_i = make_uint2(0, 0);
    uint64_t pf_top[2] = {0, 0};
    bool ok = true;

    auto prefetch = [&](int t) {
        const int x = t - 2 * qd;
        if (row_on && x >= 0 && x < W) {
            pf_y = *reinterpret_cast<const uint4*>(Y + (size_t)(Y0 + ql) * g.W + x * 16);
            {
                const unsigned long long v = load_global<unsigned long long>(Cp[ql >> 3] + (size_t)(Yc + (ql & 7)) * g.Wc + x * 8);
                pf_c = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
            }
            if (ql < DBINFO_DWORDS / 2) pf_i = *reinterpret_cast<const uint2*>(info_row + x * DBINFO_DWORDS + 2 * ql);
            if (qd == 0 && wq > 0) {
                pf_top[0] = ld_cc64(hb_in + (size_t)x * 32 + 2 * ql);
                pf_top[1] = ld_cc64(hb_in + (size_t)x * 32 + 2 * ql + 1);
            }
        }
    };

    prefetch(0);
    for (int t = 0; t < steps; ++t) {
        const int x = t - 2 * qd;
        const bool act = row_on && x >= 0 && x < W;

        // ---- quarter 0 below another wave: the records of the MB above must carry this epoch
        if (wq > 0) {
            const bool need = act && qd == 0;
            unsigned spins = 0;
            while (!__all(!need || ((pf_top[0] & 0xFFFFFFFF00000000ull) == tag &&
                                    (pf_top[1] & 0xFFFFFFFF00000000ull) == tag))) {
                __builtin_amdgcn_s_sleep(1);
                if (need) {
                    pf_top[0] = ld_cc64(hb_in + (size_t)x * 32 + 2 * ql);
                    pf_top[1] = ld_cc64(hb_in + (size_t)x * 32 + 2 * ql + 1);
                }
                if (++spins > SPIN_LIMIT) {
                    if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = false;
                    break;
                }
            }
            if (!ok) break;
        }
        // ---- assemble the tiles
        if (act) {
            *reinterpret_cast<uint4*>(&S.y[(ql + 4) * QP + LBASE + 1]) = pf_y;
            *reinterpret_cast<uint2*>(&S.c[((ql & 7) + 4) * QP + ((ql >> 3) ? CR_BASE : CB_BASE) + 1]) = pf_c;
            if (ql < DBINFO_DWORDS / 2) *reinterpret_cast<uint2*>(&S.info[2 * ql]) = pf_i;
            // a band that starts below row 0 is not filtered across its top edge (idc 1, or
            // idc 2 at a slice edge): its top-edge strengths (info dword 4) must be 0
            if (r == R0 && R0 > 0 && ql == 2 && pf_i.x != 0)
                __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (r > R0) {                                       // rows -4..-1: bottom rows of the MB above
                uint32_t v0, v1;
                if (qd == 0) { v0 = (uint32_t)pf_top[0]; v1 = (uint32_t)pf_top[1]; }
                else {
                    const uint32_t* rg = reinterpret_cast<const uint32_t*>(&L.ring[qd - 1][x & (DRING - 1)]);
                    v0 = rg[2 * ql]; v1 = rg[2 * ql + 1];
                }
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int e = 2 * ql + h;
                    const uint32_t v = h ? v1 : v0;
                    if (e < 16) S.y[(e >> 2) * QP + LBASE + 1 + (e & 3)] = v;
                    else {
                        const int k = e - 16, pl = k >> 3, i = (k >> 1) & 3, d = k & 1;
                        S.c[i * QP + (pl ? CR_BASE : CB_BASE) + 1 + d] = v;
                    }
                }
            }
        }
        if (t + 1 < steps) prefetch(t + 1);
        wave_sync();

        // ---- vertical edges: my two lines (tile rows line0, line0 + 1)
        {
            const int ra = (line0 + 4) * QP + base, rb = ra + QP;
            uint32_t A[5], Bv[5];
#pragma unroll
            for (int d = 0; d < 5; ++d) { A[d] = T[ra + d]; Bv[d] = T[rb + d]; }
            s16x2 X[20];
#pragma unroll
            for (int d = 0; d < 5; ++d) {
                X[4 * d + 0] = pair_of<0>(A[d], Bv[d]); X[4 * d + 1] = pair_of<1>(A[d], Bv[d]);
                X[4 * d + 2] = pair_of<2>(A[d], Bv[d]); X[4 * d + 3] = pair_of<3>(A[d], Bv[d]);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int bsi = luma ? k * 4 + seg : (k == 0 ? seg : (k == 1 ? 8 + seg : -1));
                const int bS = (act && bsi >= 0) ? ib[bsi] : 0;
                if (!__any(bS != 0)) continue;
                const uint32_t par = S.info[k == 0 ? pe : pi];
                const int i0 = 4 * k + 4;
                if (k == 0 && __any(bS == 4))
                    filter_edge_pk<true>(X[i0 - 4], X[i0 - 3], X[i0 - 2], X[i0 - 1], X[i0], X[i0 + 1],
                                         X[i0 + 2], X[i0 + 3], bS, par, !luma);
                else
                    filter_edge_pk<false>(X[i0 - 4], X[i0 - 3], X[i0 - 2], X[i0 - 1], X[i0], X[i0 + 1],
                                          X[i0 + 2], X[i0 + 3], bS, par, !luma);
            }
            const int nd = luma ? 5 : 3;
#pragma unroll
            for (int d = 0; d < 5; ++d) {
                if (d >= nd || !act) continue;
                T[ra + d] = dword_of<0>(X[4 * d], X[4 * d + 1], X[4 * d + 2], X[4 * d + 3]);
                T[rb + d] = dword_of<1>(X[4 * d], X[4 * d + 1], X[4 * d + 2], X[4 * d + 3]);
            }
        }
        wave_sync();

        // ---- horizontal edges: my two columns, rows -4..15 (chroma -4..7)
        {
            uint8_t* Tb = reinterpret_cast<uint8_t*>(T) + (base + 1) * 4 + line0;
            s16x2 Yv[20];
#pragma unroll
            for (int i = 0; i < 20; ++i) {
                const int row = luma ? i : min(i, CROWS - 1);
                const uint32_t v = *reinterpret_cast<const uint16_t*>(Tb + row * QP * 4);
                Yv[i] = as_s16x2(__builtin_amdgcn_perm(0u, v, 0x0c010c00u));
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int bsi = luma ? 16 + k * 4 + seg : (k == 0 ? 16 + seg : (k == 1 ? 24 + seg : -1));
                const int bS = (act && bsi >= 0) ? ib[bsi] : 0;
                if (!__any(bS != 0)) continue;
                const uint32_t par = S.info[k == 0 ? pe + 1 : pi];
                const int i0 = 4 * k + 4;
                if (k == 0 && __any(bS == 4))
                    filter_edge_pk<true>(Yv[i0 - 4], Yv[i0 - 3], Yv[i0 - 2], Yv[i0 - 1], Yv[i0], Yv[i0 + 1],
                                         Yv[i0 + 2], Yv[i0 + 3], bS, par, !luma);
                else
                    filter_edge_pk<false>(Yv[i0 - 4], Yv[i0 - 3], Yv[i0 - 2], Yv[i0 - 1], Yv[i0], Yv[i0 + 1],
                                          Yv[i0 + 2], Yv[i0 + 3], bS, par, !luma);
            }
#pragma unroll
            for (int i = 1; i < 20; ++i) {
                if (!act || (!luma && i >= CROWS)) continue;
                *reinterpret_cast<uint16_t*>(Tb + i * QP * 4) = (uint16_t)__builtin_amdgcn_perm(0u, as_u32(Yv[i]), 0x0c0c0200u);
            }
        }
        wave_sync();

        // ---- store what is final: rows -3..12 (chroma -3..4) x cols -4..11 (chroma -4..3)
        if (act) {
            const bool xl = x > 0, xr = x == W - 1;
            {                                                   // luma: lane ql -> row ql - 3
                const int row = ql - 3;
                if (row >= 0 || r > R0) {
                    const uint32_t* tr = &S.y[(row + 4) * QP + LBASE];
                    uint8_t* dst = Y + (ptrdiff_t)(Y0 + row) * g.W + x * 16;
                    if (xl) *reinterpret_cast<uint32_t*>(dst - 4) = tr[0];
                    *reinterpret_cast<uint3*>(dst) = make_uint3(tr[1], tr[2], tr[3]);
                    if (xr) *reinterpret_cast<uint32_t*>(dst + 12) = tr[4];
                }
                if (last_row && ql < 3) {                       // rows 13..15 of the last row
                    const int row2 = 13 + ql;
                    const uint32_t* tr = &S.y[(row2 + 4) * QP + LBASE];
                    uint8_t* dst = Y + (ptrdiff_t)(Y0 + row2) * g.W + x * 16;
                    if (xl) *reinterpret_cast<uint32_t*>(dst - 4) = tr[0];
                    *reinterpret_cast<uint3*>(dst) = make_uint3(tr[1], tr[2], tr[3]);
                    if (xr) *reinterpret_cast<uint32_t*>(dst + 12) = tr[4];
                }
            }
            {                                                   // chroma: lane -> plane ql >> 3, row (ql & 7) - 3
                const int pl = ql >> 3, row = (ql & 7) - 3, cb = pl ? CR_BASE : CB_BASE;
                if (row >= 0 || r > R0) {
                    const uint32_t* tr = &S.c[(row + 4) * QP + cb];
                    uint8_t* dst = Cp[pl] + (ptrdiff_t)(Yc + row) * g.Wc + x * 8;
                    if (xl) *reinterpret_cast<uint32_t*>(dst - 4) = tr[0];
                    *reinterpret_cast<uint32_t*>(dst) = tr[1];
                    if (xr) *reinterpret_cast<uint32_t*>(dst + 4) = tr[2];
                }
                if (last_row && (ql & 7) < 3) {                 // rows 5..7 of the last row
                    const int row2 = 5 + (ql & 7);
                    const uint32_t* tr = &S.c[(row2 + 4) * QP + cb];
                    uint8_t* dst = Cp[pl] + (ptrdiff_t)(Yc + row2) * g.Wc + x * 8;
                    if (xl) *reinterpret_cast<uint32_t*>(dst - 4) = tr[0];
                    *reinterpret_cast<uint32_t*>(dst) = tr[1];
                    if (xr) *reinterpret_cast<uint32_t*>(dst + 4) = tr[2];
                }
            }
            // ---- bottom rows into this quarter's ring: MB x cols 0..11 (+12..15 at the row
            // end), MB x-1 cols 12..15 (chroma: 0..3 / 4..7)
            if (feeds_ring || feeds_hb) {
                uint32_t* rg = reinterpret_cast<uint32_t*>(L.ring[qd]);
                const int ex = (x & (DRING - 1)) * 32, ep = ((x + DRING - 1) & (DRING - 1)) * 32;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int e = 2 * ql + h;
                    if (e < 16) {                               // luma row 12 + (e >> 2), dword e & 3
                        const int i = e >> 2, d = e & 3;
                        const uint32_t* tr = &S.y[(12 + i + 4) * QP + LBASE];
                        if (d < 3) rg[ex + e] = tr[1 + d];
                        else {
                            if (xl) rg[ep + e] = tr[0];
                            if (xr) rg[ex + e] = tr[4];
                        }
                    } else {
                        const int k = e - 16, pl = k >> 3, i = (k >> 1) & 3, d = k & 1;
                        const uint32_t* tr = &S.c[(4 + i + 4) * QP + (pl ? CR_BASE : CB_BASE)];
                        if (d == 0) rg[ex + e] = tr[1];
                        else {
                            if (xl) rg[ep + e] = tr[0];
                            if (xr) rg[ex + e] = tr[2];
                        }
                    }
                }
            }
        }
        wave_sync();
        // ---- last quarter: completed records (MB x-1, and MB x at the row end) to the next wave
        if (act && feeds_hb) {
            const uint32_t* rg = reinterpret_cast<const uint32_t*>(L.ring[qd]);
            const int ex = (x & (DRING - 1)) * 32, ep = ((x + DRING - 1) & (DRING - 1)) * 32;
            if (x > 0) {
                st_cc64(hb_out + (size_t)(x - 1) * 32 + 2 * ql, tag | rg[ep + 2 * ql]);
                st_cc64(hb_out + (size_t)(x - 1) * 32 + 2 * ql + 1, tag | rg[ep + 2 * ql + 1]);
            }
            if (x == W - 1) {
                st_cc64(hb_out + (size_t)x * 32 + 2 * ql, tag | rg[ex + 2 * ql]);
                st_cc64(hb_out + (size_t)x * 32 + 2 * ql + 1, tag | rg[ex + 2 * ql + 1]);
            }
        }
        // ---- carry the right four columns into the left strip: luma rows -4..15, chroma -4..7
        if (act) {
#pragma unroll
            for (int h = 0; h < 3; ++h) {
                const int e = ql + 16 * h;
                if (e < LROWS) S.y[e * QP + LBASE] = S.y[e * QP + LBASE + 4];
                else if (e < LROWS + 2 * CROWS) {
                    const int k = e - LROWS, pl = k / CROWS, row = k - pl * CROWS, cb = pl ? CR_BASE : CB_BASE;
                    S.c[row * QP + cb] = S.c[row * QP + cb + 2];
                }
            }
        }
        wave_sync();
    }
    if (!ok && feeds_hb)                                        // release the wave below (the error is flagged)
        for (int x = 0; x < W; ++x) {
            st_cc64(hb_out + (size_t)x * 32 + 2 * ql, tag);
            st_cc64(hb_out + (size_t)x * 32 + 2 * ql + 1, tag);
        }
}
