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

// pic_motion_params of a 4x4 block: ref_pic identity = DPB slot via the slice ref list
// (interpret_mb.cc:611-623), or -1 when the list is unused.
DEV MotionRef motion_at(const h264r_batch& b, const Geom& g, int pic, const h264r_mb* mbs,
                        const h264r_slice* slices, int bx4, int by4)
{
    MotionRef r;
    const size_t base = (size_t)pic * 2 * g.motion_plane;
    const int idx = by4 * g.W4 + bx4;
    const h264r_mb* mb = &mbs[(by4 >> 2) * g.wmb + (bx4 >> 2)];
    const h264r_slice* sl = &slices[mb->slice];
    for (int l = 0; l < 2; ++l) {
        int ri = b.ref_idx[base + (size_t)l * g.motion_plane + idx];
        uint32_t v = b.mv[base + (size_t)l * g.motion_plane + idx];
        r.ref[l] = ri >= 0 ? sl->ref_slot[l][ri] : -1;
        r.mvx[l] = (int16_t)(v & 0xFFFF);
        r.mvy[l] = (int16_t)(v >> 16);
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
    uint8_t bs[32];
    int8_t  qpy[3];        // QpY of Q, left MB, top MB
    int8_t  qpc[2][3];     // QpC[pl] of Q, left, top
    int8_t  off_a, off_b;  // FilterOffsetA/B of Q's slice (deblock.cc:472-473)
    uint8_t pad[5];
};
static_assert(sizeof(DbInfo) == 48, "DbInfo layout");

// Deblock::strength + strength_vertical/horizontal for MB `a` (deblock.cc:78-289).
// All lanes call; lanes 0..31 compute one strength each, lane 32 the tail.
DEV void db_info_mb(const h264r_batch& b, const Geom& g, int pic, int a, int lane, DbInfo* __restrict__ out)
{
    const int mbx = a % g.wmb, mby = a / g.wmb;
    const h264r_mb* mbs = b.mbs + (size_t)pic * g.nmb;
    const h264r_slice* slices = b.slices + (size_t)pic * b.slice_stride;
    const h264r_mb q = load_mb(&mbs[a]);
    const h264r_slice* qs = &slices[q.slice];
    const int idc = qs->deblock_idc;
    const int hasL = mbx > 0, hasU = mby > 0;
    const h264r_mb L = hasL ? load_mb(&mbs[a - 1]) : q;
    const h264r_mb U = hasU ? load_mb(&mbs[a - g.wmb]) : q;
    const int fl = idc == 0 ? hasL : (idc == 2 && hasL && L.slice == q.slice);
    const int ft = idc == 0 ? hasU : (idc == 2 && hasU && U.slice == q.slice);
    const int t8 = (q.flags & H264R_MBF_T8x8) != 0;
    if (lane < 32) {
        const int hor = lane >> 4, e = (lane >> 2) & 3, s = lane & 3;
        const int en = idc != 1 && (e == 0 ? (hor ? ft : fl) : ((e & 1) ? !t8 : 1));
        int v = 0;
        if (en) {
            const h264r_mb& P = e == 0 ? (hor ? U : L) : q;
            const int special = special_slice(slices[P.slice].slice_type) || special_slice(qs->slice_type);
            const int intra = mb_is_intra(q) || mb_is_intra(P);
            const int pskip = qs->slice_type == H264R_SLICE_P && q.mb_type == H264R_P_SKIP;
            if (!hor) {
                int blkQ = 4 * s + e, blkP = 4 * s + (e == 0 ? 3 : e - 1);
                if (special) v = e == 0 ? 4 : 3;
                else if (e > 0 && pskip) v = 0;
                else if (e == 0 && intra) v = 4;
                else if (intra) v = 3;
                else if (((q.cbp_blks >> blkQ) & 1) || ((P.cbp_blks >> blkP) & 1)) v = 2;
                else if (e > 0 && (q.mb_type == H264R_P_16x16 || q.mb_type == H264R_P_16x8)) v = 0;
                else {
                    MotionRef mq = motion_at(b, g, pic, mbs, slices, mbx * 4 + e, mby * 4 + s);
                    MotionRef mp = motion_at(b, g, pic, mbs, slices, mbx * 4 + e - 1, mby * 4 + s);
                    v = bs_compare(mq, mp);
                }
            } else {
                int blkQ = 4 * e + s, blkP = (e == 0 ? 12 : 4 * (e - 1)) + s;
                if (e == 0 && (special || intra)) v = 4;
                else if (special || intra) v = 3;
                else if (e > 0 && pskip) v = 0;
                else if (((q.cbp_blks >> blkQ) & 1) || ((P.cbp_blks >> blkP) & 1)) v = 2;
                else if (e > 0 && (q.mb_type == H264R_P_16x16 || q.mb_type == H264R_P_8x16)) v = 0;
                else {
                    MotionRef mq = motion_at(b, g, pic, mbs, slices, mbx * 4 + s, mby * 4 + e);
                    MotionRef mp = motion_at(b, g, pic, mbs, slices, mbx * 4 + s, mby * 4 + e - 1);
                    v = bs_compare(mq, mp);
                }
            }
        }
        out->bs[lane] = (uint8_t)v;
    } else if (lane == 32) {
        uint32_t w[4];
        w[0] = (uint8_t)q.qp_y | ((uint32_t)(uint8_t)L.qp_y << 8) | ((uint32_t)(uint8_t)U.qp_y << 16) |
               ((uint32_t)(uint8_t)q.qp_c[0] << 24);
        w[1] = (uint8_t)L.qp_c[0] | ((uint32_t)(uint8_t)U.qp_c[0] << 8) | ((uint32_t)(uint8_t)q.qp_c[1] << 16) |
               ((uint32_t)(uint8_t)L.qp_c[1] << 24);
        w[2] = (uint8_t)U.qp_c[1] | ((uint32_t)(uint8_t)qs->filter_offset_a << 8) |
               ((uint32_t)(uint8_t)qs->filter_offset_b << 16);
        w[3] = 0;
        *reinterpret_cast<uint4*>(&out->qpy[0]) = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

constexpr int LP = 20;   // luma tile pitch: cols -4..15
constexpr int CP = 12;   // chroma tile pitch: cols -4..7

struct alignas(16) DbLds {
    uint8_t lt[20 * LP];        // rows -4..15
    uint8_t ct[2][12 * CP];     // rows -4..7
    uint8_t bs[32];
};

// alpha/beta/tc0 for one edge (filter_edge deblock.cc:469-480), 8-bit.
DEV void edge_params(int qpp, int qpq, int offa, int offb, int& alpha, int& beta, int& idxA)
{
    int qPav = (qpp + qpq + 1) >> 1;
    idxA = clip3(0, 51, qPav + offa);
    int idxB = clip3(0, 51, qPav + offb);
    alpha = DB_AB[idxA] & 255;
    beta = (DB_AB[idxB] >> 8) & 255;
}

DEV int tc0_of(int idxA, int bS) { return bS < 4 ? (int)((DB_TC0[idxA] >> (8 * (bS - 1))) & 255) : 0; }

// Filter one line of N samples held in registers across the edges of one direction.
// NE edges, edge k at v[4k+4] (q0); bs[k] its strength; qpp/qpq/params per edge.
template <int NE, int N>
DEV void filter_line(int (&v)[N], const int* bs, const int* alpha, const int* beta, const int* idxA, int chroma)
{
#pragma unroll
    for (int k = 0; k < NE; ++k) {
        if (!bs[k]) continue;
        filter_samples(v[4 * k + 0], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3],
                       v[4 * k + 4], v[4 * k + 5], v[4 * k + 6], v[4 * k + 7],
                       alpha[k], beta[k], bs[k], chroma, tc0_of(idxA[k], bs[k]));
    }
}

// Deblock MB (mbx, mby) of picture `pic`: vertical then horizontal edges
// (filter_vertical / filter_horizontal deblock.cc:488-535); one wave.  Every MB
// that precedes it in raster order and shares samples with it -- (x-1,y),
// (x,y-1), (x+1,y-1) -- must already be filtered.
DEV void deblock_mb(const h264r_batch& b, const Geom& g, int pic, int mbx, int mby, int lane, DbLds& S,
                    const DbInfo* __restrict__ info_all)
{
    const int a = mby * g.wmb + mbx;
    const DbInfo* info = info_all + (size_t)pic * g.nmb + a;
    const int hasL = mbx > 0, hasU = mby > 0;
    uint8_t* Y = b.out_y + (size_t)pic * g.ysz;
    uint8_t* Cpl[2] = {b.out_u + (size_t)pic * g.csz, b.out_v + (size_t)pic * g.csz};
    const int X0 = mbx * 16, Y0 = mby * 16, Xc = mbx * 8, Yc = mby * 8;

    // ---- stage: strengths + samples (dword loads; rows/cols -4..-1 where a neighbour exists)
    if (lane < 8) reinterpret_cast<uint32_t*>(S.bs)[lane] = reinterpret_cast<const uint32_t*>(info->bs)[lane];
    for (int k = lane; k < 100; k += 64) {
        int r = k / 5, d = k % 5;
        if ((r < 4 && !hasU) || (d == 0 && !hasL)) continue;
        reinterpret_cast<uint32_t*>(S.lt)[k] =
            *reinterpret_cast<const uint32_t*>(Y + (size_t)(Y0 + r - 4) * g.W + X0 - 4 + 4 * d);
    }
    for (int k = lane; k < 72; k += 64) {
        int pl = k / 36, r = (k % 36) / 3, d = k % 3;
        if ((r < 4 && !hasU) || (d == 0 && !hasL)) continue;
        reinterpret_cast<uint32_t*>(S.ct[pl])[r * 3 + d] =
            *reinterpret_cast<const uint32_t*>(Cpl[pl] + (size_t)(Yc + r - 4) * g.Wc + Xc - 4 + 4 * d);
    }
    const uint4 tail = *reinterpret_cast<const uint4*>(&info->qpy[0]);
    const int qpyQ = (int8_t)(tail.x & 255), qpyL = (int8_t)((tail.x >> 8) & 255), qpyU = (int8_t)((tail.x >> 16) & 255);
    const int qpc[2][3] = {{(int8_t)(tail.x >> 24), (int8_t)(tail.y & 255), (int8_t)((tail.y >> 8) & 255)},
                           {(int8_t)((tail.y >> 16) & 255), (int8_t)(tail.y >> 24), (int8_t)(tail.z & 255)}};
    const int offa = (int8_t)((tail.z >> 8) & 255), offb = (int8_t)((tail.z >> 16) & 255);
    wave_sync();

    for (int hor = 0; hor < 2; ++hor) {
        if (lane < 16) {                                       // luma line `lane`
            int bs[4], al[4], be[4], ia[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                bs[e] = S.bs[hor * 16 + e * 4 + (lane >> 2)];
                edge_params(e == 0 ? (hor ? qpyU : qpyL) : qpyQ, qpyQ, offa, offb, al[e], be[e], ia[e]);
            }
            int v[20];
            if (!hor) {
                const uint32_t* row = reinterpret_cast<const uint32_t*>(S.lt + (lane + 4) * LP);
#pragma unroll
                for (int d = 0; d < 5; ++d) {
                    uint32_t w = row[d];
#pragma unroll
                    for (int k = 0; k < 4; ++k) v[4 * d + k] = (w >> (8 * k)) & 255;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 20; ++i) v[i] = S.lt[i * LP + lane + 4];
            }
            filter_line<4>(v, bs, al, be, ia, 0);
            if (!hor) {
                uint32_t* row = reinterpret_cast<uint32_t*>(S.lt + (lane + 4) * LP);
#pragma unroll
                for (int d = 0; d < 5; ++d)
                    row[d] = (uint32_t)v[4 * d] | ((uint32_t)v[4 * d + 1] << 8) | ((uint32_t)v[4 * d + 2] << 16) |
                             ((uint32_t)v[4 * d + 3] << 24);
            } else {
#pragma unroll
                for (int i = 1; i < 20; ++i) S.lt[i * LP + lane + 4] = (uint8_t)v[i];
            }
        } else if (lane < 32) {                                // chroma line
            const int pl = (lane - 16) >> 3, r = (lane - 16) & 7;
            uint8_t* ct = S.ct[pl];
            int bs[2], al[2], be[2], ia[2];
#pragma unroll
            for (int ce = 0; ce < 2; ++ce) {
                bs[ce] = S.bs[hor * 16 + (ce ? 2 : 0) * 4 + (r >> 1)];     // StrengthIdx = pel << 1 (:460)
                edge_params(ce == 0 ? qpc[pl][hor ? 2 : 1] : qpc[pl][0], qpc[pl][0], offa, offb, al[ce], be[ce], ia[ce]);
            }
            int v[12];
            if (!hor) {
                const uint32_t* row = reinterpret_cast<const uint32_t*>(ct + (r + 4) * CP);
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    uint32_t w = row[d];
#pragma unroll
                    for (int k = 0; k < 4; ++k) v[4 * d + k] = (w >> (8 * k)) & 255;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 12; ++i) v[i] = ct[i * CP + r + 4];
            }
            filter_line<2>(v, bs, al, be, ia, 1);
            if (!hor) {
                uint32_t* row = reinterpret_cast<uint32_t*>(ct + (r + 4) * CP);
#pragma unroll
                for (int d = 0; d < 3; ++d)
                    row[d] = (uint32_t)v[4 * d] | ((uint32_t)v[4 * d + 1] << 8) | ((uint32_t)v[4 * d + 2] << 16) |
                             ((uint32_t)v[4 * d + 3] << 24);
            } else {
#pragma unroll
                for (int i = 1; i < 12; ++i) ct[i * CP + r + 4] = (uint8_t)v[i];
            }
        }
        wave_sync();
    }

    // ---- write back: rows -3..15 (top rows only if the top MB exists), dwords from col -4
    for (int k = lane; k < 95; k += 64) {
        int r = k / 5 + 1, d = k % 5;
        if ((r < 4 && !hasU) || (d == 0 && !hasL)) continue;
        *reinterpret_cast<uint32_t*>(Y + (size_t)(Y0 + r - 4) * g.W + X0 - 4 + 4 * d) =
            reinterpret_cast<const uint32_t*>(S.lt)[r * 5 + d];
    }
    for (int k = lane; k < 66; k += 64) {
        int pl = k / 33, r = (k % 33) / 3 + 1, d = k % 3;
        if ((r < 4 && !hasU) || (d == 0 && !hasL)) continue;
        *reinterpret_cast<uint32_t*>(Cpl[pl] + (size_t)(Yc + r - 4) * g.Wc + Xc - 4 + 4 * d) =
            reinterpret_cast<const uint32_t*>(S.ct[pl])[r * 3 + d];
    }
}

}  // namespace h264r
