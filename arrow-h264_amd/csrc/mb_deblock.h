// mb_deblock.h -- in-loop deblocking filter of one MB (one wave), gfx950.
//
// The reference filters MBs in raster order, vertical edges then horizontal
// edges per MB (Deblock::deblock_pic, deblock.cc:537-552), and the result is
// order-dependent: MB (x,y)'s top edge reads samples MB (x+1,y-1)'s left edge
// wrote.  MBs on one anti-diagonal x + 2y == step are independent, so each
// k_picture walks them with per-row progress counters (one wave per MB row).
// Boundary strengths are computed in the same wave (strength* deblock.cc:78-289,
// bs_compare_mvs :40-75), the samples are staged in LDS, filtered row-per-lane
// (vertical edges) and column-per-lane (horizontal edges) with filter_strong /
// filter_normal (deblock.cc:327-415), and written back.
#pragma once
#include "device_common.h"
#include "launch_cfg.h"

namespace h264r {


struct MotionRef {
    int ref[2];
    int mvx[2], mvy[2];
};

// Per-4x4-block motion as resolved in k_inter4 (block_motion): {mv, ref_idx | slot << 8} per list.
// ref identity = DPB slot of RefPicList[l][ref_idx] (pic_motion_params::ref_pic,
// interpret_mb.cc:611-623) with the field parity bit (H264R_REF_BOTTOM: the two fields of a
// frame are different pictures), -1 when the list is unused.
DEV MotionRef motion_of(uint2 w0, uint2 w1)
{
    MotionRef r;
    const uint2 w[2] = {w0, w1};
#pragma unroll
    for (int l = 0; l < 2; ++l) {
        const int ri = (int8_t)(w[l].y & 255), slot = (int8_t)((w[l].y >> 8) & 255);
        r.ref[l] = ri >= 0 ? slot : -1;
        r.mvx[l] = (int16_t)(w[l].x & 0xFFFF);
        r.mvy[l] = (int16_t)(w[l].x >> 16);
    }
    return r;
}

// mvlimit 4 in frame pictures, 2 in field pictures (deblock.cc:35-38, 86, 164)
DEV int cmp_mv(const MotionRef& a, int la, const MotionRef& c, int lc, int mvlim)
{
    return (int)(iabs(a.mvx[la] - c.mvx[lc]) >= 4) | (int)(iabs(a.mvy[la] - c.mvy[lc]) >= mvlim);
}

DEV int bs_compare(const MotionRef& p, const MotionRef& q, int mvlim)   // deblock.cc:40-75
{
    int p0 = p.ref[0], q0 = q.ref[0], p1 = p.ref[1], q1 = q.ref[1];
    if ((p0 == q0 && p1 == q1) || (p0 == q1 && p1 == q0)) {
        if (p0 != p1) {
            if (p0 == q0) return cmp_mv(p, 0, q, 0, mvlim) | cmp_mv(p, 1, q, 1, mvlim);
            return cmp_mv(p, 0, q, 1, mvlim) | cmp_mv(p, 1, q, 0, mvlim);
        }
        return (cmp_mv(p, 0, q, 0, mvlim) | cmp_mv(p, 1, q, 1, mvlim)) & (cmp_mv(p, 0, q, 1, mvlim) | cmp_mv(p, 1, q, 0, mvlim));
    }
    return 1;
}

DEV int special_slice(int t) { return t == H264R_SLICE_SP || t == H264R_SLICE_SI; }

// Per-MB deblocking record, produced by k_inter for every MB (fully parallel) so
// that the order-dependent walk only loads 48 bytes per MB.  bs[] folds the edge
// enables of Deblock::strength (deblock.cc:236-278) into the strengths: a
// disabled edge has bS 0.  bs[hor * 16 + edge * 4 + segment]; chroma edge 0 uses
// luma edge 0, chroma edge 1 (sample 4) luma edge 2 (deblock.cc:430-433).
struct DbInfo {
    uint8_t  bs[32];
    uint32_t par[9];       // [Y, Cb, Cr][left edge, top edge, internal edges]: edge_word()
    uint32_t pad[3];
};
static_assert(sizeof(DbInfo) == 80, "DbInfo layout");
constexpr int DBINFO_DWORDS = 20;
constexpr int DEBLOCK2_UNITS = 64 / H264R_DB2_LPU;   // k_deblock2: (picture, MB row) units per wave

// alpha | beta << 8 | tc0(bS 1..3) << 16 / 21 / 26 for one edge: filter_edge
// deblock.cc:469-480 (qPav of the two MBs' QPs, indexA/B with MbQ's slice offsets),
// 8-bit tables (Tables 8-16 / 8-17, deblock.cc:294-324).
// ab / tc0: DB_AB / DB_TC0 or a copy of them (k_inter4r keeps one in LDS: read from global
// memory, the lookup was a dependent round trip per 16-MB group)
DEV uint32_t edge_word(int qpp, int qpq, int offa, int offb, const uint32_t* ab = DB_AB, const uint32_t* tc0 = DB_TC0)
{
    const int qPav = (qpp + qpq + 1) >> 1;
    const int idxA = clip3(0, 51, qPav + offa), idxB = clip3(0, 51, qPav + offb);
    const uint32_t t = tc0[idxA];
    return (ab[idxA] & 255) | (ab[idxB] & 0xFF00) | ((t & 31) << 16) | (((t >> 8) & 31) << 21) |
           (((t >> 16) & 31) << 26);
}
struct DbTables {
    uint32_t ab[52], tc0[52];
};
// thread t < 52 copies entry t (the workgroup has >= 52 threads): load, then store, so a
// caller can issue its own loads between the two
DEV uint2 db_tables_load(int t) { const int i = min(t, 51); return make_uint2(DB_AB[i], DB_TC0[i]); }
DEV void db_tables_store(DbTables& T, int t, uint2 v)
{
    if (t < 52) { T.ab[t] = v.x; T.tc0[t] = v.y; }
}

constexpr int TP = 5;     // tile pitch in dwords: left margin + 16 samples
constexpr int TR = 20;    // tile rows: -4..15 (chroma uses -4..7)

// Bottom rows of one MB for the row below: luma rows 12..15 (4 x 4 dwords) and
// chroma rows 4..7 (2 planes x 4 x 2 dwords) -- 128 bytes, one cache line.
struct alignas(16) RingEntry {
    uint32_t y[4][4];
    uint32_t c[2][4][2];
};
static_assert(sizeof(RingEntry) == 128, "RingEntry is one 128-B line");

// One MB row's working set in LDS: three tiles of identical geometry (Y, Cb, Cr;
// [row + 4][dword], dword 0 = the 4 samples left of the MB) and the MB's DbInfo.
// The shared geometry lets luma and chroma lanes run the same instructions.
struct alignas(16) DbLds {
    uint32_t t[3][TR * TP];
    uint32_t info[DBINFO_DWORDS];
    uint32_t zero;                // bS 0 of the edges a chroma line does not have
};

// One edge of one line, branch-free (filter_strong / filter_normal,
// deblock.cc:327-415, as chosen by filter_edge :459-485): s[i0-4..i0+3] are
// p3..p0 q0..q3; bS 0 leaves the line unchanged.  `par` is the edge's
// edge_word(); chroma lines use tc0 + 1 and never touch p1/q1 or the strong
// 3-tap outputs.
template <bool STRONG>
DEV void filter_edge_line(int& p3, int& p2, int& p1, int& p0, int& q0, int& q1, int& q2, int& q3, int bS,
                          uint32_t par, bool chroma)
{
    const int alpha = par & 255, beta = (par >> 8) & 255;
    // every candidate computed, then selected: the compiler otherwise sinks each into a
    // lane-divergent branch of its own (bS and the decisions differ between a wave's lines)
    int tc0r = (int)((par >> (11 + 5 * min(max(bS, 1), 3))) & 31);
    asm volatile("" : "+v"(tc0r));
    const int tc0 = (bS >= 1 && bS <= 3) ? tc0r : 0;
    // all four tests evaluated (a short-circuit && on lane-varying operands becomes branches)
    const bool filt = ((int)(bS != 0) & (int)(iabs(p0 - q0) < alpha) & (int)(iabs(p1 - p0) < beta) &
                       (int)(iabs(q1 - q0) < beta)) != 0;
    const bool apb = iabs(p2 - p0) < beta, aqb = iabs(q2 - q0) < beta;
    // bS < 4 (filter_normal)
    const int tc = tc0 + (chroma ? 1 : (int)apb + (int)aqb);
    const int delta = clip3(-tc, tc, ((q0 - p0) * 4 + (p1 - q1) + 4) >> 3);
    const int avg = (p0 + q0 + 1) >> 1;
    const int n_p0 = clip255(p0 + delta), n_q0 = clip255(q0 - delta);
    int t_p1 = p1 + clip3(-tc0, tc0, (p2 + avg - p1 * 2) >> 1), t_q1 = q1 + clip3(-tc0, tc0, (q2 + avg - q1 * 2) >> 1);
    asm volatile("" : "+v"(t_p1), "+v"(t_q1));
    const int n_p1 = (!chroma && apb) ? t_p1 : p1;
    const int n_q1 = (!chroma && aqb) ? t_q1 : q1;
    if (!STRONG) {            // no lane of the wave has bS 4 on this edge
        p1 = filt ? n_p1 : p1; p0 = filt ? n_p0 : p0; q0 = filt ? n_q0 : q0; q1 = filt ? n_q1 : q1;
        return;
    }
    // bS == 4 (filter_strong)
    const bool strong = iabs(p0 - q0) < ((alpha >> 2) + 2);
    const bool sp = !chroma && apb && strong, sq = !chroma && aqb && strong;
    int a_p0 = (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3, b_p0 = (2 * p1 + p0 + q1 + 2) >> 2;
    int a_p1 = (p2 + p1 + p0 + q0 + 2) >> 2, a_p2 = (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3;
    int a_q0 = (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3, b_q0 = (2 * q1 + q0 + p1 + 2) >> 2;
    int a_q1 = (p0 + q0 + q1 + q2 + 2) >> 2, a_q2 = (2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3;
    asm volatile("" : "+v"(a_p0), "+v"(b_p0), "+v"(a_p1), "+v"(a_p2), "+v"(a_q0), "+v"(b_q0), "+v"(a_q1), "+v"(a_q2));
    const int s_p0 = sp ? a_p0 : b_p0, s_p1 = sp ? a_p1 : p1, s_p2 = sp ? a_p2 : p2;
    const int s_q0 = sq ? a_q0 : b_q0, s_q1 = sq ? a_q1 : q1, s_q2 = sq ? a_q2 : q2;
    const bool is4 = bS == 4, f4 = filt && is4, fn = filt && !is4;
    p2 = f4 ? s_p2 : p2; p1 = f4 ? s_p1 : (fn ? n_p1 : p1); p0 = f4 ? s_p0 : (fn ? n_p0 : p0);
    q0 = f4 ? s_q0 : (fn ? n_q0 : q0); q1 = f4 ? s_q1 : (fn ? n_q1 : q1); q2 = f4 ? s_q2 : q2;
}

// The two filter passes of one MB on the LDS tiles: vertical edges with one lane per
// sample row, then horizontal edges with one lane per column (filter_vertical /
// filter_horizontal deblock.cc:488-535).  Lanes 0..15 luma lines, 16..31 chroma
// lines (Cb 16..23, Cr 24..31) run the same 4-edge code: a chroma line has its
// edges at samples 0 and 4 (chroma edge 1 takes the bS of luma edge 2,
// StrengthIdx = pel << 1, deblock.cc:430-433, :460) and bS 0 on the other two.
// Edges no lane of the wave filters are skipped.  Every lane of the wave calls, and
// separates the two passes (and whatever it does between them) with wave_sync().
DEV void filter_pass(DbLds& S, int lane, const int hor)
{
    const bool luma = lane < 16;
    const int pl = luma ? 0 : 1 + ((lane - 16) >> 3), li = luma ? lane : (lane - 16) & 7;
    const int seg = luma ? li >> 2 : li >> 1;
    uint32_t* T = S.t[pl];
    uint8_t* Tb = reinterpret_cast<uint8_t*>(T);
    const uint8_t* ib = reinterpret_cast<const uint8_t*>(S.info);
    const int zoff = (int)(reinterpret_cast<const uint8_t*>(&S.zero) - ib);
    // byte offsets of this line's bS per edge (before + hor * 16), parameter words
    int bso[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) bso[k] = luma ? k * 4 + seg : (k == 0 ? seg : (k == 1 ? 8 + seg : -1));
    const int pe = luma ? 8 : 11 + 3 * (pl - 1), pi = luma ? 10 : 13 + 3 * (pl - 1);
    {
        int bsk[4];
        uint32_t park[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            bsk[k] = ib[bso[k] >= 0 ? bso[k] + hor * 16 : zoff];
            park[k] = S.info[k == 0 ? pe + hor : pi];
        }
        int v[20];
        if (!hor) {
#pragma unroll
            for (int d = 0; d < 5; ++d) {
                const uint32_t w = T[(li + 4) * TP + d];
#pragma unroll
                for (int c = 0; c < 4; ++c) v[4 * d + c] = (w >> (8 * c)) & 255;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 20; ++i) v[i] = Tb[i * TP * 4 + li + 4];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (!__any(bsk[k] != 0)) continue;
            const int i0 = 4 * k + 4;
            if (k == 0 && __any(bsk[k] == 4))
                filter_edge_line<true>(v[i0 - 4], v[i0 - 3], v[i0 - 2], v[i0 - 1], v[i0], v[i0 + 1], v[i0 + 2], v[i0 + 3],
                                       bsk[k], park[k], !luma);
            else
                filter_edge_line<false>(v[i0 - 4], v[i0 - 3], v[i0 - 2], v[i0 - 1], v[i0], v[i0 + 1], v[i0 + 2], v[i0 + 3],
                                        bsk[k], park[k], !luma);
        }
        if (!hor) {
#pragma unroll
            for (int d = 0; d < 5; ++d)
                T[(li + 4) * TP + d] = (uint32_t)v[4 * d] | ((uint32_t)v[4 * d + 1] << 8) |
                                       ((uint32_t)v[4 * d + 2] << 16) | ((uint32_t)v[4 * d + 3] << 24);
        } else {
#pragma unroll
            for (int i = 1; i < 20; ++i) Tb[i * TP * 4 + li + 4] = (uint8_t)v[i];
        }
    }
}

}  // namespace h264r
