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

namespace h264r {


struct MotionRef {
    int ref[2];
    int mvx[2], mvy[2];
};

// Per-4x4-block motion as resolved by k_prep: {mv, ref_idx | slot << 8} per list.
// ref identity = DPB slot of RefPicList[l][ref_idx] (pic_motion_params::ref_pic,
// interpret_mb.cc:611-623), -1 when the list is unused.
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

DEV int cmp_mv(const MotionRef& a, int la, const MotionRef& c, int lc)   // deblock.cc:35-38 (frame: mvlimit 4)
{
    return (int)(iabs(a.mvx[la] - c.mvx[lc]) >= 4) | (int)(iabs(a.mvy[la] - c.mvy[lc]) >= 4);
}

DEV int bs_compare(const MotionRef& p, const MotionRef& q)              // deblock.cc:40-75
{
    int p0 = p.ref[0], q0 = q.ref[0], p1 = p.ref[1], q1 = q.ref[1];
    if ((p0 == q0 && p1 == q1) || (p0 == q1 && p1 == q0)) {
        if (p0 != p1) {
            if (p0 == q0) return cmp_mv(p, 0, q, 0) | cmp_mv(p, 1, q, 1);
            return cmp_mv(p, 0, q, 1) | cmp_mv(p, 1, q, 0);
        }
        return (cmp_mv(p, 0, q, 0) | cmp_mv(p, 1, q, 1)) & (cmp_mv(p, 0, q, 1) | cmp_mv(p, 1, q, 0));
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

// alpha | beta << 8 | tc0(bS 1..3) << 16 / 21 / 26 for one edge: filter_edge
// deblock.cc:469-480 (qPav of the two MBs' QPs, indexA/B with MbQ's slice offsets),
// 8-bit tables (Tables 8-16 / 8-17, deblock.cc:294-324).
DEV uint32_t edge_word(int qpp, int qpq, int offa, int offb)
{
    const int qPav = (qpp + qpq + 1) >> 1;
    const int idxA = clip3(0, 51, qPav + offa), idxB = clip3(0, 51, qPav + offb);
    const uint32_t t = DB_TC0[idxA];
    return (DB_AB[idxA] & 255) | (DB_AB[idxB] & 0xFF00) | ((t & 31) << 16) | (((t >> 8) & 31) << 21) |
           (((t >> 16) & 31) << 26);
}

// Deblock::strength + strength_vertical/horizontal for MB `a` (deblock.cc:78-289).
// All lanes call; lanes 0..31 compute one strength each, lanes 32..40 the edge
// parameters (alpha/beta/tc0 per plane and edge class).  `mot`
// is the picture's resolved motion (k_prep), [list][H4][W4]; every load is issued
// before the first decision so the record and motion latencies overlap.
DEV void db_info_mb(const h264r_batch& b, const Geom& g, int pic, int a, int lane, const uint2* __restrict__ mot,
                    DbInfo* __restrict__ out)
{
    const int mbx = a % g.wmb, mby = a / g.wmb;
    const h264r_mb* mbs = b.mbs + (size_t)pic * g.nmb;
    const h264r_slice* slices = b.slices + (size_t)pic * b.slice_stride;
    const int hor = (lane >> 4) & 1, e = (lane >> 2) & 3, s = lane & 3;
    const int qx = mbx * 4 + (hor ? s : e), qy = mby * 4 + (hor ? e : s);
    const int px = max(qx - (hor ? 0 : 1), 0), py = max(qy - (hor ? 1 : 0), 0);
    const uint2 q0 = mot[qy * g.W4 + qx], q1 = mot[g.motion_plane + qy * g.W4 + qx];
    const uint2 p0 = mot[py * g.W4 + px], p1 = mot[g.motion_plane + py * g.W4 + px];
    const h264r_mb q = load_mb(&mbs[a]);
    const int hasL = mbx > 0, hasU = mby > 0;
    const h264r_mb L = load_mb(&mbs[hasL ? a - 1 : a]);
    const h264r_mb U = load_mb(&mbs[hasU ? a - g.wmb : a]);
    const h264r_slice* qs = &slices[q.slice];
    const int idc = qs->deblock_idc;
    const int fl = idc == 0 ? hasL : (idc == 2 && hasL && L.slice == q.slice);
    const int ft = idc == 0 ? hasU : (idc == 2 && hasU && U.slice == q.slice);
    const int t8 = (q.flags & H264R_MBF_T8x8) != 0;
    if (lane < 32) {
        const int en = idc != 1 && (e == 0 ? (hor ? ft : fl) : ((e & 1) ? !t8 : 1));
        int v = 0;
        if (en) {
            const h264r_mb& P = e == 0 ? (hor ? U : L) : q;
            const int special = special_slice(slices[P.slice].slice_type) || special_slice(qs->slice_type);
            const int intra = mb_is_intra(q) || mb_is_intra(P);
            const int pskip = qs->slice_type == H264R_SLICE_P && q.mb_type == H264R_P_SKIP;
            const int blkQ = hor ? 4 * e + s : 4 * s + e;
            const int blkP = hor ? (e == 0 ? 12 : 4 * (e - 1)) + s : 4 * s + (e == 0 ? 3 : e - 1);
            const int coded = ((q.cbp_blks >> blkQ) & 1) || ((P.cbp_blks >> blkP) & 1);
            const int same_part = e > 0 && (q.mb_type == H264R_P_16x16 ||
                                            q.mb_type == (hor ? H264R_P_8x16 : H264R_P_16x8));
            if (!hor) {
                if (special) v = e == 0 ? 4 : 3;
                else if (e > 0 && pskip) v = 0;
                else if (e == 0 && intra) v = 4;
                else if (intra) v = 3;
                else if (coded) v = 2;
                else if (same_part) v = 0;
                else v = bs_compare(motion_of(q0, q1), motion_of(p0, p1));
            } else {
                if (e == 0 && (special || intra)) v = 4;
                else if (special || intra) v = 3;
                else if (e > 0 && pskip) v = 0;
                else if (coded) v = 2;
                else if (same_part) v = 0;
                else v = bs_compare(motion_of(q0, q1), motion_of(p0, p1));
            }
        }
        out->bs[lane] = (uint8_t)v;
    } else if (lane < 32 + 9) {                        // edge parameters
        const int k = lane - 32, pl = k / 3, which = k - pl * 3;
        const int qyP = which == 0 ? L.qp_y : (which == 1 ? U.qp_y : q.qp_y);
        const int qcP0 = which == 0 ? L.qp_c[0] : (which == 1 ? U.qp_c[0] : q.qp_c[0]);
        const int qcP1 = which == 0 ? L.qp_c[1] : (which == 1 ? U.qp_c[1] : q.qp_c[1]);
        const int qq = pl == 0 ? q.qp_y : (pl == 1 ? q.qp_c[0] : q.qp_c[1]);
        const int qp = pl == 0 ? qyP : (pl == 1 ? qcP0 : qcP1);
        out->par[k] = edge_word(qp, qq, qs->filter_offset_a, qs->filter_offset_b);
    }
}

constexpr int LP = 20;    // luma tile: rows -4..15 x cols -4..15, 5 dwords per row
constexpr int CP = 12;    // chroma tile: rows -4..7 x cols -4..7, 3 dwords per row

// Bottom rows of one MB for the row below: luma rows 12..15 (4 x 4 dwords) and
// chroma rows 4..7 (2 planes x 4 x 2 dwords) -- 128 bytes, one cache line.
struct alignas(16) RingEntry {
    uint32_t y[4][4];
    uint32_t c[2][4][2];
};
static_assert(sizeof(RingEntry) == 128, "RingEntry is one 128-B line");

// One MB row's working set in LDS: the MB being filtered plus its 4-sample
// left/top margins, and its deblocking record.
struct alignas(16) DbLds {
    uint32_t lt[20 * 5];          // luma tile, [row + 4][dword]
    uint32_t ct[2][12 * 3];       // chroma tiles
    uint32_t info[DBINFO_DWORDS]; // the MB's DbInfo
};

DEV uint8_t* ltb(DbLds& S) { return reinterpret_cast<uint8_t*>(S.lt); }
DEV uint8_t* ctb(DbLds& S, int pl) { return reinterpret_cast<uint8_t*>(S.ct[pl]); }

// Filter one line held as packed bytes w[0..NE] (4 samples per dword; edge k sits
// between dword k and dword k+1) across NE edges; edges are sequential because
// neighbouring edges share samples (deblock.cc:459-485 per edge, :495-502 order).
template <int NE>
DEV void filter_line_packed(uint32_t (&w)[NE + 1], const uint8_t* bsrow, int seg, uint32_t par0, uint32_t pari,
                            int chroma, int bsidx_step)
{
#pragma unroll
    for (int k = 0; k < NE; ++k) {
        const int bS = bsrow[k * bsidx_step * 4 + seg];
        if (!bS) continue;
        const uint32_t par = k == 0 ? par0 : pari;
        const int alpha = par & 255, beta = (par >> 8) & 255;
        const int tc0 = bS < 4 ? (int)((par >> (16 + 5 * (bS - 1))) & 31) : 0;
        const uint32_t a = w[k], c = w[k + 1];
        int p3 = a & 255, p2 = (a >> 8) & 255, p1 = (a >> 16) & 255, p0 = a >> 24;
        int q0 = c & 255, q1 = (c >> 8) & 255, q2 = (c >> 16) & 255, q3 = c >> 24;
        filter_samples(p3, p2, p1, p0, q0, q1, q2, q3, alpha, beta, bS, chroma, tc0);
        w[k] = (uint32_t)p3 | ((uint32_t)p2 << 8) | ((uint32_t)p1 << 16) | ((uint32_t)p0 << 24);
        w[k + 1] = (uint32_t)q0 | ((uint32_t)q1 << 8) | ((uint32_t)q2 << 16) | ((uint32_t)q3 << 24);
    }
}

// The two filter passes of one MB on the LDS tiles: vertical edges with one lane per
// sample row, then horizontal edges with one lane per column (filter_vertical /
// filter_horizontal deblock.cc:488-535).  Lanes 0..15 luma, 16..31 chroma;
// every lane of the wave calls (the passes are separated by wave_sync).
DEV void filter_mb(DbLds& S, int lane, bool act)
{
    const uint8_t* bs = reinterpret_cast<const uint8_t*>(S.info);
#pragma unroll 1
    for (int hor = 0; hor < 2; ++hor) {
        if (!act) {
        } else if (lane < 16) {
            uint32_t w[5];
            uint8_t* lt = ltb(S);
            if (!hor) {
#pragma unroll
                for (int d = 0; d < 5; ++d) w[d] = S.lt[(lane + 4) * 5 + d];
            } else {
#pragma unroll
                for (int d = 0; d < 5; ++d)
                    w[d] = (uint32_t)lt[(4 * d) * LP + lane + 4] | ((uint32_t)lt[(4 * d + 1) * LP + lane + 4] << 8) |
                           ((uint32_t)lt[(4 * d + 2) * LP + lane + 4] << 16) | ((uint32_t)lt[(4 * d + 3) * LP + lane + 4] << 24);
            }
            filter_line_packed<4>(w, &bs[hor * 16], lane >> 2, S.info[8 + hor], S.info[10], 0, 1);
            if (!hor) {
#pragma unroll
                for (int d = 0; d < 5; ++d) S.lt[(lane + 4) * 5 + d] = w[d];
            } else {
#pragma unroll
                for (int i = 1; i < 20; ++i) lt[i * LP + lane + 4] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
            }
        } else if (lane < 32) {
            const int pl = (lane - 16) >> 3, r = (lane - 16) & 7;
            uint32_t w[3];
            uint8_t* ct = ctb(S, pl);
            if (!hor) {
#pragma unroll
                for (int d = 0; d < 3; ++d) w[d] = S.ct[pl][(r + 4) * 3 + d];
            } else {
#pragma unroll
                for (int d = 0; d < 3; ++d)
                    w[d] = (uint32_t)ct[(4 * d) * CP + r + 4] | ((uint32_t)ct[(4 * d + 1) * CP + r + 4] << 8) |
                           ((uint32_t)ct[(4 * d + 2) * CP + r + 4] << 16) | ((uint32_t)ct[(4 * d + 3) * CP + r + 4] << 24);
            }
            // chroma edge 1 uses luma edge 2 (bsidx_step 2); StrengthIdx = pel << 1 (deblock.cc:460)
            filter_line_packed<2>(w, &bs[hor * 16], r >> 1, S.info[11 + 3 * pl + hor], S.info[13 + 3 * pl], 1, 2);
            if (!hor) {
#pragma unroll
                for (int d = 0; d < 3; ++d) S.ct[pl][(r + 4) * 3 + d] = w[d];
            } else {
#pragma unroll
                for (int i = 1; i < 12; ++i) ct[i * CP + r + 4] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
            }
        }
        wave_sync();
    }
}

}  // namespace h264r
