// k_deblock.hip -- in-loop deblocking filter for gfx950.
//
// The reference filters MBs in raster order, vertical edges then horizontal
// edges per MB (Deblock::deblock_pic, deblock.cc:537-552), and the result is
// order-dependent: MB (x,y)'s top edge reads samples MB (x+1,y-1)'s left edge
// wrote.  MBs on one anti-diagonal x + 2y == step are independent, so each
// launch filters one diagonal of every picture of the batch (one wave per MB).
// Boundary strengths are computed in the same wave (strength* deblock.cc:78-289,
// bs_compare_mvs :40-75), the samples are staged in LDS, filtered row-per-lane
// (vertical edges) and column-per-lane (horizontal edges) with filter_strong /
// filter_normal (deblock.cc:327-415), and written back.
#include "device_common.h"

using namespace h264r;

namespace {

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

constexpr int LP = 20;   // luma tile pitch: cols -4..15
constexpr int CP = 12;   // chroma tile pitch: cols -4..7

struct DbLds {
    uint8_t lt[20 * LP];        // rows -4..15
    uint8_t ct[2][12 * CP];     // rows -4..7
    uint8_t bs[2][4][4];        // [0 vertical / 1 horizontal][edge][segment]
};

}  // namespace

extern "C" __global__ __launch_bounds__(64) void k_deblock(h264r_batch b, int step)
{
    __shared__ DbLds S;
    const int pic = blockIdx.y, lane = threadIdx.x;
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    int y0 = step - (g.wmb - 1) > 0 ? (step - (g.wmb - 1) + 1) / 2 : 0;
    const int mby = y0 + blockIdx.x, mbx = step - 2 * mby;
    if (mby >= g.hmb || mbx < 0 || mbx >= g.wmb) return;
    const int a = mby * g.wmb + mbx;
    const h264r_mb* mbs = b.mbs + (size_t)pic * g.nmb;
    const h264r_slice* slices = b.slices + (size_t)pic * b.slice_stride;
    const h264r_mb q = load_mb(&mbs[a]);
    const h264r_slice* qs = &slices[q.slice];
    const int idc = qs->deblock_idc;
    if (idc == 1) return;                                      // deblock.cc:236, 494, 512

    // ---- edge flags (Deblock::strength deblock.cc:236-278)
    const int hasL = mbx > 0, hasU = mby > 0;
    const h264r_mb L = hasL ? load_mb(&mbs[a - 1]) : q;
    const h264r_mb U = hasU ? load_mb(&mbs[a - g.wmb]) : q;
    const int fl = idc == 0 ? hasL : (hasL && L.slice == q.slice);
    const int ft = idc == 0 ? hasU : (hasU && U.slice == q.slice);
    const int t8 = (q.flags & H264R_MBF_T8x8) != 0;
    // luma edge e enabled: e==0 -> fl/ft, e==1,3 -> !t8, e==2 -> 1; chroma: edges 0 (fl/ft) and 1 (internal)

    // ---- boundary strengths: lanes 0..15 vertical (edge, row group), 16..31 horizontal
    if (lane < 32) {
        const int hor = lane >> 4, e = (lane >> 2) & 3, s = lane & 3;
        const int en = e == 0 ? (hor ? ft : fl) : ((e & 1) ? !t8 : 1);
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
        S.bs[hor][e][s] = (uint8_t)v;
    }

    // ---- stage samples (rows/cols -4..-1 only where a neighbour MB exists)
    uint8_t* Y = b.out_y + (size_t)pic * g.ysz;
    uint8_t* Cpl[2] = {b.out_u + (size_t)pic * g.csz, b.out_v + (size_t)pic * g.csz};
    const int X0 = mbx * 16, Y0 = mby * 16, Xc = mbx * 8, Yc = mby * 8;
    for (int k = lane; k < 20 * 20; k += 64) {
        int y = k / 20 - 4, x = k % 20 - 4;
        if ((x < 0 && !hasL) || (y < 0 && !hasU)) continue;
        S.lt[(y + 4) * LP + x + 4] = Y[(size_t)(Y0 + y) * g.W + X0 + x];
    }
    for (int k = lane; k < 2 * 144; k += 64) {
        int pl = k / 144, r = k % 144, y = r / 12 - 4, x = r % 12 - 4;
        if ((x < 0 && !hasL) || (y < 0 && !hasU)) continue;
        S.ct[pl][(y + 4) * CP + x + 4] = Cpl[pl][(size_t)(Yc + y) * g.Wc + Xc + x];
    }
    __syncthreads();

    // ---- per-edge filter parameters (filter_edge deblock.cc:469-480)
    auto params = [&](int qpp, int qpq, int& alpha, int& beta, int& idxA) {
        int qPav = (qpp + qpq + 1) >> 1;
        idxA = clip3(0, 51, qPav + qs->filter_offset_a);
        int idxB = clip3(0, 51, qPav + qs->filter_offset_b);
        alpha = DB_AB[idxA] & 255;
        beta = (DB_AB[idxB] >> 8) & 255;
    };

    // ---- vertical edges: lane = sample row (filter_vertical deblock.cc:488-504)
    for (int pass = 0; pass < 2; ++pass) {
        const int hor = pass;
        if (lane < 16) {                                      // luma row/column `lane`
            int v[20];
            for (int i = 0; i < 20; ++i) v[i] = hor ? S.lt[i * LP + lane + 4] : S.lt[(lane + 4) * LP + i];
            for (int e = 0; e < 4; ++e) {
                int bS = S.bs[hor][e][lane >> 2];
                int en = e == 0 ? (hor ? ft : fl) : ((e & 1) ? !t8 : 1);
                if (!en || !bS) continue;
                const h264r_mb& P = e == 0 ? (hor ? U : L) : q;
                int alpha, beta, ia;
                params(P.qp_y, q.qp_y, alpha, beta, ia);
                int tc0 = bS < 4 ? (int)((DB_TC0[ia] >> (8 * (bS - 1))) & 255) : 0;
                int* w = &v[4 * e];
                filter_samples(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], alpha, beta, bS, 0, tc0);
            }
            for (int i = 1; i < 20; ++i) {
                if (hor) S.lt[i * LP + lane + 4] = (uint8_t)v[i];
                else S.lt[(lane + 4) * LP + i] = (uint8_t)v[i];
            }
        } else if (lane < 32) {                               // chroma rows/columns
            const int pl = (lane - 16) >> 3, r = (lane - 16) & 7;
            uint8_t* ct = S.ct[pl];
            int v[12];
            for (int i = 0; i < 12; ++i) v[i] = hor ? ct[i * CP + r + 4] : ct[(r + 4) * CP + i];
            for (int ce = 0; ce < 2; ++ce) {
                int bS = S.bs[hor][ce ? 2 : 0][(2 * r) >> 2];     // StrengthIdx = pel << 1 (:460)
                int en = ce == 0 ? (hor ? ft : fl) : 1;
                if (!en || !bS) continue;
                const h264r_mb& P = ce == 0 ? (hor ? U : L) : q;
                int alpha, beta, ia;
                params(P.qp_c[pl], q.qp_c[pl], alpha, beta, ia);
                int tc0 = bS < 4 ? (int)((DB_TC0[ia] >> (8 * (bS - 1))) & 255) : 0;
                int* w = &v[4 * ce];
                filter_samples(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], alpha, beta, bS, 1, tc0);
            }
            for (int i = 1; i < 12; ++i) {
                if (hor) ct[i * CP + r + 4] = (uint8_t)v[i];
                else ct[(r + 4) * CP + i] = (uint8_t)v[i];
            }
        }
        __syncthreads();
    }

    // ---- write back what this MB may have modified (rows/cols -3..15, not the corner)
    for (int k = lane; k < 19 * 19; k += 64) {
        int y = k / 19 - 3, x = k % 19 - 3;
        if ((x < 0 && !fl) || (y < 0 && !ft) || (x < 0 && y < 0)) continue;
        Y[(size_t)(Y0 + y) * g.W + X0 + x] = S.lt[(y + 4) * LP + x + 4];
    }
    for (int k = lane; k < 2 * 121; k += 64) {
        int pl = k / 121, r = k % 121, y = r / 11 - 3, x = r % 11 - 3;
        if ((x < 0 && !fl) || (y < 0 && !ft) || (x < 0 && y < 0)) continue;
        Cpl[pl][(size_t)(Yc + y) * g.Wc + Xc + x] = S.ct[pl][(y + 4) * CP + x + 4];
    }
}
