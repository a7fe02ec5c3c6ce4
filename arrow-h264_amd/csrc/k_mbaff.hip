// k_mbaff.hip -- MBAFF frames (mb_adaptive_frame_field_flag) on the reconstruction path, gfx950.
//
// An MBAFF frame codes each MB pair as two frame MBs or as two field MBs (H264R_MBF_FIELD,
// include/h264r.h).  The reference decodes the pairs in MB-address order into the MB-contiguous
// layout, interleaves the field MBs (MbAffPostProc deblock.cc:581-620) and then filters
// (deblock.cc:622-656); its intra prediction and its loop filter find every neighbouring sample
// through Neighbour::get_location / get_neighbour (neighbour.cc:47-227), i.e. the geometric sample
// of the frame and the MB holding it.  These kernels write the frame as it is after MbAffPostProc
// and address it geometrically (H/ = R/src/codec/h264/):
//
//   k_mbaff_inter    one workgroup per MB, every MB of every picture at once: I_PCM and inter MBs
//                    (residual + motion compensation; a field MB predicts from the FIELDS of its
//                    list's frames, get_ref_pic dpb.cc:1046-1055, with field block rows and the
//                    chroma parity offset, inter_prediction.cc:356-361,470-474).
//   k_mbaff_intra    one workgroup per MB pair, launched per anti-diagonal d = x + 2 y of the pair
//                    grid: a pair's intra neighbours lie in the pairs left, above-left, above and
//                    above-right, all on earlier diagonals.  The pair and its border (34 x 25 luma,
//                    2 x 18 x 9 chroma samples) are staged in LDS; the top MB, then the bottom MB,
//                    each 4x4 / 8x8 block in turn (intra_prediction.cc:137-894), from a table of
//                    the MB's outside neighbours looked up once per MB (nb_table).
//   k_mbaff_deblock  one wave per MB pair, per anti-diagonal: Deblock::strength for the pair's two
//                    MBs, then filter_vertical / filter_horizontal of the top MB and of the bottom
//                    MB (deblock.cc:78-535) on an LDS tile of the pair and the samples its edges
//                    reach (8 rows above, 4 columns left).  A pair on diagonal d modifies only
//                    itself, its left pair (d - 1) and its upper pair (d - 2); the pairs that
//                    modify it come later, so every diagonal sees the samples the reference's
//                    MB-order walk sees.
//
// This is the MBAFF format's own launch sequence: the frame / field-picture path (k_inter4r,
// k_intra_levels, k_deblock2) keeps its layout.  4:2:0 only; no SP slices, lossless MBs or
// implicit weights (the host refuses them).
#include "device_common.h"

namespace h264r {
namespace {

// ------------------------------------------------------------------ picture views
struct MPic {
    const h264r_mb* mbs;
    const uint32_t* mv;
    const int8_t* ref;
    const h264r_slice* sl;
    const h264r_quant* q;
    const uint8_t* const* tab;
    uint8_t* out[3];
    int wmb, hmb, W4, mplane;
    int cip;
};

DEV MPic mpic(const h264r_batch& b, int p)
{
    MPic P;
    const size_t nmb = (size_t)b.width_mbs * b.height_mbs;
    P.wmb = b.width_mbs; P.hmb = b.height_mbs; P.W4 = 4 * b.width_mbs;
    P.mplane = P.W4 * 4 * b.height_mbs;
    P.mbs = b.mbs + (size_t)p * nmb;
    P.mv = b.mv + (size_t)p * 2 * P.mplane;
    P.ref = b.ref_idx + (size_t)p * 2 * P.mplane;
    P.sl = b.slices + (size_t)p * b.slice_stride;
    P.q = b.quant + p;
    P.tab = b.ref_planes + (b.ref_planes_stride ? (size_t)p * b.ref_planes_stride : 0);
    P.out[0] = b.out_y + (size_t)p * nmb * 256;
    P.out[1] = b.out_u + (size_t)p * nmb * 64;
    P.out[2] = b.out_v + (size_t)p * nmb * 64;
    P.cip = b.pics[p].constrained_intra_pred;
    return P;
}

DEV bool is_fld(const MPic& P, int r) { return (P.mbs[r].flags & H264R_MBF_FIELD) != 0; }

// Neighbour::get_location (neighbour.cc:47-77): frame position of sample (ox, oy) of MB r (storage
// index, include/h264r.h), on the luma (16 x 16) or the 4:2:0 chroma grid (8 x 8)
DEV void mloc(const MPic& P, int r, int maxW, int maxH, int ox, int oy, int& x, int& y)
{
    const int mby = r / P.wmb, bb = mby & 1;
    x = (r % P.wmb) * maxW + ox;
    y = (mby >> 1) * 2 * maxH + (is_fld(P, r) ? bb + 2 * oy : bb * maxH + oy);
}

// Neighbour::get_mb / get_neighbour (neighbour.cc:175-227): the MB holding frame sample (x, y), or -1
DEV int mmb_at(const MPic& P, int maxW, int maxH, int x, int y, int* ly)
{
    if (x < 0 || x >= P.wmb * maxW || y < 0 || y >= P.hmb * maxH) return -1;
    const int top = ((y / (2 * maxH)) * 2) * P.wmb + x / maxW, r = y % (2 * maxH);
    const bool f = is_fld(P, top);
    const int bb = f ? (y & 1) : (r >= maxH);
    if (ly) *ly = f ? r / 2 : r % maxH;
    return top + bb * P.wmb;
}

DEV int maddr(const MPic& P, int r)            // MB address of storage index r
{
    const int mby = r / P.wmb;
    return 2 * ((mby >> 1) * P.wmb + r % P.wmb) + (mby & 1);
}

// ------------------------------------------------------------------ residual (256 threads)
struct ResLds {
    int cof[3][256];       // dequantised coefficients, then the residual (luma 16 x 16, chroma 8 x 8)
    int tmp[3][256];
};

DEV void idct8_1d(const int in[8], int out[8])                  // transform.cc:658-683
{
    const int e0 = in[0] + in[4], e1 = -in[3] + in[5] - in[7] - (in[7] >> 1);
    const int e2 = in[0] - in[4], e3 = in[1] + in[7] - in[3] - (in[3] >> 1);
    const int e4 = (in[2] >> 1) - in[6], e5 = -in[1] + in[7] + in[5] + (in[5] >> 1);
    const int e6 = in[2] + (in[6] >> 1), e7 = in[3] + in[5] + in[1] + (in[1] >> 1);
    const int f0 = e0 + e6, f1 = e1 + (e7 >> 2), f2 = e2 + e4, f3 = e3 + (e5 >> 2);
    const int f4 = e2 - e4, f5 = (e3 >> 2) - e5, f6 = e0 - e6, f7 = e7 - (e1 >> 2);
    out[0] = f0 + f7; out[1] = f2 + f5; out[2] = f4 + f3; out[3] = f6 + f1;
    out[4] = f6 - f1; out[5] = f4 - f3; out[6] = f2 - f5; out[7] = f0 - f7;
}

// coeff_* + inverse_quantize, transform_luma_dc / transform_chroma_dc, inverse_4x4 / inverse_8x8
// (transform.cc:394-456, 460-733, 825-910) of one 4:2:0 MB: R.cof holds its residual on return.
// Blocks the cbp leaves uncoded have zero coefficients, so their residual is zero and
// clip(residual + prediction) is the prediction (construction transform.cc:913-984).
DEV void mb_residual(const h264r_mb& m, const int16_t* lv, const h264r_quant& q, ResLds& R, int t)
{
    for (int k = t; k < 3 * 256; k += 256) (&R.cof[0][0])[k] = 0;
    __syncthreads();
    const int cbpl = m.cbp & 15, cbpc = m.cbp >> 4;
    const int inter = (m.flags & H264R_MBF_INTRA) ? 0 : 1;
    const bool t8 = (m.flags & H264R_MBF_T8x8) != 0, i16 = m.mb_type == H264R_I_16x16;
    const int nb8 = __popc(cbpl);
    const int16_t* cac = lv + 64 * nb8;                              // include/h264r.h level layout
    const int16_t* ldc = cac + (cbpc == 2 ? 128 : 0);
    const int16_t* cdc = ldc + (i16 ? 16 : 0);
    {
        const int b8 = t >> 6, k = t & 63;
        if ((cbpl >> b8) & 1) {
            const int lev = lv[__popc(cbpl & ((1 << b8) - 1)) * 64 + k];
            const int qp = m.qp_scaled[0], per = qp / 6, rem = qp % 6;
            if (lev) {
                if (!t8) {
                    const int b4 = k >> 4, pos = k & 15;
                    if (!(i16 && pos == 0)) {
                        const int bx = (b8 & 1) * 2 + (b4 & 1), by = (b8 >> 1) * 2 + (b4 >> 1);
                        R.cof[0][(by * 4 + pos / 4) * 16 + bx * 4 + pos % 4] =
                            ((lev * q.scale4x4[inter][0][rem][pos]) * (1 << per) + 8) >> 4;
                    }
                } else {
                    const int x0 = (b8 & 1) * 8, y0 = (b8 >> 1) * 8;
                    R.cof[0][(y0 + k / 8) * 16 + x0 + k % 8] = ((lev * q.scale8x8[inter][0][rem][k]) * (1 << per) + 32) >> 6;
                }
            }
        }
    }
    if (t < 128 && cbpc == 2) {                                        // chroma AC
        const int pl = 1 + (t >> 6), k = t & 63, b = k >> 4, pos = k & 15;
        const int lev = pos ? cac[(pl - 1) * 64 + b * 16 + pos] : 0;
        if (lev) {
            const int qP = m.qp_scaled[pl];
            R.cof[pl][((b / 2) * 4 + pos / 4) * 8 + (b % 2) * 4 + pos % 4] =
                ((lev * q.scale4x4[inter][pl][qP % 6][pos]) * (1 << (qP / 6)) + 8) >> 4;
        }
    }
    if (t == 200 && i16) {                                             // luma DC (transform.cc:515-554, 825-856)
        int c[4][4], e[4][4];
        const int qP = m.qp_scaled[0], scale = q.scale4x4[0][0][qP % 6][0];
        for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) c[i][j] = ldc[i * 4 + j];
        for (int i = 0; i < 4; ++i) {
            const int d0 = c[i][0] + c[i][2], d1 = c[i][0] - c[i][2], d2 = c[i][1] - c[i][3], d3 = c[i][1] + c[i][3];
            e[i][0] = d0 + d3; e[i][1] = d1 + d2; e[i][2] = d1 - d2; e[i][3] = d0 - d3;
        }
        for (int j = 0; j < 4; ++j) {
            const int h0 = e[0][j] + e[2][j], h1 = e[0][j] - e[2][j], h2 = e[1][j] - e[3][j], h3 = e[1][j] + e[3][j];
            const int f[4] = {h0 + h3, h1 + h2, h1 - h2, h0 - h3};
            for (int i = 0; i < 4; ++i)
                R.cof[0][(i * 4) * 16 + j * 4] = qP >= 36 ? (f[i] * scale) * (1 << (qP / 6 - 6))
                                                          : (f[i] * scale + (1 << (5 - qP / 6))) >> (6 - qP / 6);
        }
    }
    if ((t == 201 || t == 202) && cbpc) {                              // chroma DC (transform.cc:460-481, 858-889)
        const int pl = t - 200, qP = m.qp_scaled[pl], scale = q.scale4x4[inter][pl][qP % 6][0];
        const int16_t* c = cdc + (pl - 1) * 4;
        const int f[4] = {c[0] + c[1] + c[2] + c[3], c[0] - c[1] + c[2] - c[3], c[0] + c[1] - c[2] - c[3], c[0] - c[1] - c[2] + c[3]};
        for (int k = 0; k < 4; ++k) R.cof[pl][((k >> 1) * 4) * 8 + (k & 1) * 4] = ((f[k] * scale) * (1 << (qP / 6))) >> 5;
    }
    __syncthreads();
    // row passes
    if (t8) {
        if (t < 32) {
            const int bk = t >> 3, i = t & 7, x0 = (bk & 1) * 8, y0 = (bk >> 1) * 8;
            int in[8], o[8];
            for (int k = 0; k < 8; ++k) in[k] = R.cof[0][(y0 + i) * 16 + x0 + k];
            idct8_1d(in, o);
            for (int k = 0; k < 8; ++k) R.tmp[0][(y0 + i) * 16 + x0 + k] = o[k];
        }
    } else if (t < 64) {
        const int bk = t >> 2, i = t & 3, x0 = (bk & 3) * 4, y0 = (bk >> 2) * 4;
        const int* d = &R.cof[0][(y0 + i) * 16 + x0];
        const int e0 = d[0] + d[2], e1 = d[0] - d[2], e2 = (d[1] >> 1) - d[3], e3 = d[1] + (d[3] >> 1);
        int* o = &R.tmp[0][(y0 + i) * 16 + x0];
        o[0] = e0 + e3; o[1] = e1 + e2; o[2] = e1 - e2; o[3] = e0 - e3;
    }
    if (t >= 64 && t < 96) {
        const int u = t - 64, pl = 1 + (u >> 4), bk = (u >> 2) & 3, i = u & 3, x0 = (bk & 1) * 4, y0 = (bk >> 1) * 4;
        const int* d = &R.cof[pl][(y0 + i) * 8 + x0];
        const int e0 = d[0] + d[2], e1 = d[0] - d[2], e2 = (d[1] >> 1) - d[3], e3 = d[1] + (d[3] >> 1);
        int* o = &R.tmp[pl][(y0 + i) * 8 + x0];
        o[0] = e0 + e3; o[1] = e1 + e2; o[2] = e1 - e2; o[3] = e0 - e3;
    }
    __syncthreads();
    // column passes (into cof: the residual)
    if (t8) {
        if (t < 32) {
            const int bk = t >> 3, j = t & 7, x0 = (bk & 1) * 8, y0 = (bk >> 1) * 8;
            int in[8], o[8];
            for (int k = 0; k < 8; ++k) in[k] = R.tmp[0][(y0 + k) * 16 + x0 + j];
            idct8_1d(in, o);
            for (int k = 0; k < 8; ++k) R.cof[0][(y0 + k) * 16 + x0 + j] = (o[k] + 32) >> 6;
        }
    } else if (t < 64) {
        const int bk = t >> 2, j = t & 3, x0 = (bk & 3) * 4, y0 = (bk >> 2) * 4;
        const int f0 = R.tmp[0][(y0 + 0) * 16 + x0 + j], f1 = R.tmp[0][(y0 + 1) * 16 + x0 + j];
        const int f2 = R.tmp[0][(y0 + 2) * 16 + x0 + j], f3 = R.tmp[0][(y0 + 3) * 16 + x0 + j];
        const int g0 = f0 + f2, g1 = f0 - f2, g2 = (f1 >> 1) - f3, g3 = f1 + (f3 >> 1);
        R.cof[0][(y0 + 0) * 16 + x0 + j] = (g0 + g3 + 32) >> 6;
        R.cof[0][(y0 + 1) * 16 + x0 + j] = (g1 + g2 + 32) >> 6;
        R.cof[0][(y0 + 2) * 16 + x0 + j] = (g1 - g2 + 32) >> 6;
        R.cof[0][(y0 + 3) * 16 + x0 + j] = (g0 - g3 + 32) >> 6;
    }
    if (t >= 64 && t < 96) {
        const int u = t - 64, pl = 1 + (u >> 4), bk = (u >> 2) & 3, j = u & 3, x0 = (bk & 1) * 4, y0 = (bk >> 1) * 4;
        const int f0 = R.tmp[pl][(y0 + 0) * 8 + x0 + j], f1 = R.tmp[pl][(y0 + 1) * 8 + x0 + j];
        const int f2 = R.tmp[pl][(y0 + 2) * 8 + x0 + j], f3 = R.tmp[pl][(y0 + 3) * 8 + x0 + j];
        const int g0 = f0 + f2, g1 = f0 - f2, g2 = (f1 >> 1) - f3, g3 = f1 + (f3 >> 1);
        R.cof[pl][(y0 + 0) * 8 + x0 + j] = (g0 + g3 + 32) >> 6;
        R.cof[pl][(y0 + 1) * 8 + x0 + j] = (g1 + g2 + 32) >> 6;
        R.cof[pl][(y0 + 2) * 8 + x0 + j] = (g1 - g2 + 32) >> 6;
        R.cof[pl][(y0 + 3) * 8 + x0 + j] = (g0 - g3 + 32) >> 6;
    }
    __syncthreads();
}

// ------------------------------------------------------------------ motion compensation
DEV int rpx(const uint8_t* img, int W, int pitch, int H, int x, int y)
{
    return img[clip3(0, H - 1, y) * pitch + clip3(0, W - 1, x)];
}
DEV int tap6(int a, int b, int c, int d, int e, int f) { return a - 5 * b + 20 * c + 20 * d - 5 * e + f; }

// one luma sample of get_block_luma (inter_prediction.cc:158-340) on a clamped view of the
// reference (its pads replaced by clamping, as in the frame path)
DEV int luma_mc(const uint8_t* img, int W, int pitch, int H, int x, int y, int xf, int yf)
{
#define S(dx, dy) rpx(img, W, pitch, H, x + (dx), y + (dy))
#define B1(dy) tap6(S(-2, dy), S(-1, dy), S(0, dy), S(1, dy), S(2, dy), S(3, dy))
#define H1(dx) tap6(S(dx, -2), S(dx, -1), S(dx, 0), S(dx, 1), S(dx, 2), S(dx, 3))
    if (xf == 0 && yf == 0) return S(0, 0);
    if (yf == 0) {
        const int b = clip255((B1(0) + 16) >> 5);
        return xf == 2 ? b : (S(xf == 1 ? 0 : 1, 0) + b + 1) >> 1;
    }
    if (xf == 0) {
        const int h = clip255((H1(0) + 16) >> 5);
        return yf == 2 ? h : (S(0, yf == 1 ? 0 : 1) + h + 1) >> 1;
    }
    if ((xf & 1) && (yf & 1)) {
        const int bb = clip255((B1(yf == 3 ? 1 : 0) + 16) >> 5);
        const int hh = clip255((H1(xf == 3 ? 1 : 0) + 16) >> 5);
        return (bb + hh + 1) >> 1;
    }
    const int j = clip255((tap6(B1(-2), B1(-1), B1(0), B1(1), B1(2), B1(3)) + 512) >> 10);
    if (xf == 2 && yf == 2) return j;
    if (xf == 2) return (j + clip255((B1(yf == 3 ? 1 : 0) + 16) >> 5) + 1) >> 1;
    return (j + clip255((H1(xf == 3 ? 1 : 0) + 16) >> 5) + 1) >> 1;
#undef S
#undef B1
#undef H1
}

DEV int chroma_mc(const uint8_t* img, int W, int pitch, int H, int xi, int yi, int xf, int yf)   // :380-404
{
    const int A = rpx(img, W, pitch, H, xi, yi), B = rpx(img, W, pitch, H, xi + 1, yi);
    const int Cc = rpx(img, W, pitch, H, xi, yi + 1), D = rpx(img, W, pitch, H, xi + 1, yi + 1);
    return ((8 - xf) * (8 - yf) * A + xf * (8 - yf) * B + (8 - xf) * yf * Cc + xf * yf * D + 32) >> 6;
}

DEV int rshift_rnd(int x, int a) { return a > 0 ? (x + (1 << (a - 1))) >> a : x * (1 << -a); }   // inter_prediction.cc:35-38

// the prediction of sample (x, y) of plane pl of inter MB r (inter_pred, mc_prediction,
// bi_prediction, inter_prediction.cc:53-156, 448-536)
DEV int inter_sample(const MPic& P, int r, int pl, int x, int y, int* err)
{
    const h264r_mb m = P.mbs[r];
    const h264r_slice& sl = P.sl[m.slice];
    const int mbx = r % P.wmb, mby = r / P.wmb;
    const bool fmb = (m.flags & H264R_MBF_FIELD) != 0;
    const int mbot = mby & 1;
    const int i = pl ? x >> 1 : x >> 2, j = pl ? y >> 1 : y >> 2;           // the sample's 4x4 luma block
    const int idx = (mby * 4 + j) * P.W4 + mbx * 4 + i;
    const int row4 = fmb ? (mby >> 1) * 4 : mby * 4;                       // block_y_aff (:470-474)
    const int Wp = pl ? P.wmb * 8 : P.wmb * 16, Hp = pl ? P.hmb * 8 : P.hmb * 16;
    int v[2] = {0, 0}, rw[2] = {-1, -1};
    for (int l = 0; l < 2; ++l) {
        const int rr = P.ref[l * P.mplane + idx];
        if (rr < 0) continue;
        rw[l] = fmb ? rr >> 1 : rr;
        const int slot = rw[l] < H264R_MAX_REFS ? sl.ref_slot[l][rw[l]] : -1;
        const uint8_t* base = slot >= 0 && slot < H264R_MAX_SLOTS ? P.tab[slot * 3 + pl] : nullptr;
        if (!base) { __hip_atomic_store(err, 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); continue; }
        const uint32_t mvw = P.mv[l * P.mplane + idx];
        const int vx = (mbx * 4 + i) * 16 + (int16_t)(mvw & 0xFFFF);
        const int vy = (row4 + j) * 16 + (int16_t)(mvw >> 16);
        const int bot = fmb && ((rr & 1) != mbot);                         // get_ref_pic
        const uint8_t* img = base + bot * Wp;
        const int pitch = fmb ? 2 * Wp : Wp, Hv = fmb ? Hp >> 1 : Hp;
        if (!pl) v[l] = luma_mc(img, Wp, pitch, Hv, (vx >> 2) + (x & 3), (vy >> 2) + (y & 3), vx & 3, vy & 3);
        else {
            const int vyc = vy + (fmb && bot != mbot ? (mbot ? 2 : -2) : 0);   // :356-361
            v[l] = chroma_mc(img, Wp, pitch, Hv, (vx >> 3) + (x & 1), (vyc >> 3) + (y & 1), vx & 7, vyc & 7);
        }
    }
    const int dir = (rw[0] >= 0 && rw[1] >= 0) ? 2 : rw[0] >= 0 ? 0 : 1;
    if (dir != 2) {
        if (sl.wp_mode == 1) {
            const int w = sl.wp_weight[dir][rw[dir]][pl], o = sl.wp_offset[dir][rw[dir]][pl];
            return clip255(rshift_rnd(w * v[dir], pl ? sl.chroma_log2_wd : sl.luma_log2_wd) + o);
        }
        return v[dir];
    }
    if (sl.wp_mode == 1) {
        const int w0 = sl.wp_weight[0][rw[0]][pl], w1 = sl.wp_weight[1][rw[1]][pl];
        const int o = (sl.wp_offset[0][rw[0]][pl] + sl.wp_offset[1][rw[1]][pl] + 1) >> 1;
        return clip255(rshift_rnd(w0 * v[0] + w1 * v[1], (pl ? sl.chroma_log2_wd : sl.luma_log2_wd) + 1) + o);
    }
    return (v[0] + v[1] + 1) >> 1;
}

// ------------------------------------------------------------------ intra prediction
// Neighbour sample of MB r as get_neighbour + the ctor's slice check find it (intra_prediction.cc:
// 145-152): its MB (-1 = not available) and its place in the pair tile
DEV int nbr(const MPic& P, int r, int maxW, int maxH, int ox, int oy, int px, int py, int& tx, int& ty)
{
    int gx, gy;
    mloc(P, r, maxW, maxH, ox, oy, gx, gy);
    tx = gx - px * maxW; ty = gy - py * 2 * maxH;
    const int n = mmb_at(P, maxW, maxH, gx, gy, nullptr);
    if (n < 0 || n == r) return n;
    return maddr(P, n) < maddr(P, r) && P.mbs[n].slice == P.mbs[r].slice ? n : -1;
}
DEV bool intra_ok(const MPic& P, int n) { return n >= 0 && (!P.cip || (P.mbs[n].flags & H264R_MBF_INTRA)); }

// luma tile: rows -2 .. 31, columns -1 .. 23 of the pair; chroma: rows -2 .. 15, columns -1 .. 7
constexpr int TYW = 25, TYH = 34, TCW = 9, TCH = 18;
// The neighbours of the MB being predicted, looked up once per MB (one lane each) instead of per
// block: tile index and availability (bit 0 get_neighbour found it in the slice, bit 1 also usable
// under constrained_intra_pred) of the left column, the top row, the top-right and top-left samples
// (luma), and of the chroma left column, top row and top-left sample.
struct NbTab {
    int16_t lpos[16], tpos, trpos, tlpos, clpos[8], ctpos, ctlpos;
    uint8_t lav[16], tav, trav, tlav, clav[8], ctav, ctlav;
};
struct IntraLds {
    uint8_t ty[TYH * TYW];
    uint8_t tc[2][TCH * TCW];
    ResLds R;
    NbTab nb;
};
DEV uint8_t& TY(IntraLds& L, int x, int y) { return L.ty[(y + 2) * TYW + x + 1]; }
DEV uint8_t& TC(IntraLds& L, int pl, int x, int y) { return L.tc[pl][(y + 2) * TCW + x + 1]; }

// p(x, y) of an N x N block (N 4 or 8; x in -1 .. 2N - 1, y in -1 .. N - 1), p(-1, -1) at [0]
struct Nbr { int s[26]; int av[4]; };
#define PX(n, x, y) ((y) < 0 ? (n).s[1 + (x)] : (n).s[17 + (y)])

// Intra8x8::filtering (intra_prediction.cc:413-447)
DEV void filter_8x8(const Nbr& n, Nbr& f)
{
    const int aA = n.av[0], aB = n.av[1], aD = n.av[3];
    f = n;
    if (aB) {
        f.s[1] = aD ? (n.s[0] + 2 * n.s[1] + n.s[2] + 2) >> 2 : (3 * n.s[1] + n.s[2] + 2) >> 2;
        for (int x = 1; x < 15; ++x) f.s[1 + x] = (n.s[x] + 2 * n.s[1 + x] + n.s[2 + x] + 2) >> 2;
        f.s[16] = (n.s[15] + 3 * n.s[16] + 2) >> 2;
    }
    if (aD) {
        if (aA && aB) f.s[0] = (n.s[1] + 2 * n.s[0] + n.s[17] + 2) >> 2;
        else if (aB) f.s[0] = (3 * n.s[0] + n.s[1] + 2) >> 2;
        else if (aA) f.s[0] = (3 * n.s[0] + n.s[17] + 2) >> 2;
    }
    if (aA) {
        f.s[17] = aD ? (n.s[0] + 2 * n.s[17] + n.s[18] + 2) >> 2 : (3 * n.s[17] + n.s[18] + 2) >> 2;
        for (int y = 1; y < 7; ++y) f.s[17 + y] = (n.s[16 + y] + 2 * n.s[17 + y] + n.s[18 + y] + 2) >> 2;
        f.s[24] = (n.s[23] + 3 * n.s[24] + 2) >> 2;
    }
}

// Intra4x4 / Intra8x8 modes (intra_prediction.cc:189-346, 449-606) at (x, y) of an N x N block
DEV int pred_nxn(const Nbr& n, int N, int mode, int x, int y)
{
    switch (mode) {
    case 0: return PX(n, x, -1);
    case 1: return PX(n, -1, y);
    case 2: {
        const int aA = n.av[0], aB = n.av[1];
        if (!aA && !aB) return 128;
        int sum = 0;
        if (aA) for (int k = 0; k < N; ++k) sum += PX(n, -1, k);
        if (aB) for (int k = 0; k < N; ++k) sum += PX(n, k, -1);
        const int sh = N == 4 ? 1 : 2;
        return (sum + (aA ? N / 2 : 0) + (aB ? N / 2 : 0)) >> (sh + aA + aB);
    }
    case 3:
        if (x == N - 1 && y == N - 1) return (PX(n, 2 * N - 2, -1) + 3 * PX(n, 2 * N - 1, -1) + 2) >> 2;
        return (PX(n, x + y, -1) + 2 * PX(n, x + y + 1, -1) + PX(n, x + y + 2, -1) + 2) >> 2;
    case 4:
        if (x > y) return (PX(n, x - y - 2, -1) + 2 * PX(n, x - y - 1, -1) + PX(n, x - y, -1) + 2) >> 2;
        if (x < y) return (PX(n, -1, y - x - 2) + 2 * PX(n, -1, y - x - 1) + PX(n, -1, y - x) + 2) >> 2;
        return (PX(n, 0, -1) + 2 * PX(n, -1, -1) + PX(n, -1, 0) + 2) >> 2;
    case 5: {
        const int z = 2 * x - y;
        if (z >= 0 && (z & 1) == 0) return (PX(n, x - (y >> 1) - 1, -1) + PX(n, x - (y >> 1), -1) + 1) >> 1;
        if (z >= 0) return (PX(n, x - (y >> 1) - 2, -1) + 2 * PX(n, x - (y >> 1) - 1, -1) + PX(n, x - (y >> 1), -1) + 2) >> 2;
        if (z == -1) return (PX(n, -1, 0) + 2 * PX(n, -1, -1) + PX(n, 0, -1) + 2) >> 2;
        return (PX(n, -1, y - 2 * x - 1) + 2 * PX(n, -1, y - 2 * x - 2) + PX(n, -1, y - 2 * x - 3) + 2) >> 2;
    }
    case 6: {
        const int z = 2 * y - x;
        if (z >= 0 && (z & 1) == 0) return (PX(n, -1, y - (x >> 1) - 1) + PX(n, -1, y - (x >> 1)) + 1) >> 1;
        if (z >= 0) return (PX(n, -1, y - (x >> 1) - 2) + 2 * PX(n, -1, y - (x >> 1) - 1) + PX(n, -1, y - (x >> 1)) + 2) >> 2;
        if (z == -1) return (PX(n, -1, 0) + 2 * PX(n, -1, -1) + PX(n, 0, -1) + 2) >> 2;
        return (PX(n, x - 2 * y - 1, -1) + 2 * PX(n, x - 2 * y - 2, -1) + PX(n, x - 2 * y - 3, -1) + 2) >> 2;
    }
    case 7:
        if ((y & 1) == 0) return (PX(n, x + (y >> 1), -1) + PX(n, x + (y >> 1) + 1, -1) + 1) >> 1;
        return (PX(n, x + (y >> 1), -1) + 2 * PX(n, x + (y >> 1) + 1, -1) + PX(n, x + (y >> 1) + 2, -1) + 2) >> 2;
    default: {                                                        // 8: horizontal up
        const int z = x + 2 * y, zl = 2 * N - 3;
        if (z < zl && (z & 1) == 0) return (PX(n, -1, y + (x >> 1)) + PX(n, -1, y + (x >> 1) + 1) + 1) >> 1;
        if (z < zl) return (PX(n, -1, y + (x >> 1)) + 2 * PX(n, -1, y + (x >> 1) + 1) + PX(n, -1, y + (x >> 1) + 2) + 2) >> 2;
        if (z == zl) return (PX(n, -1, N - 2) + 3 * PX(n, -1, N - 1) + 2) >> 2;
        return PX(n, -1, N - 1);
    }
    }
}

// fill L.nb for MB r of pair (px, py) (lanes 0..28; the caller synchronises)
DEV void nb_table(const MPic& P, IntraLds& L, int r, int px, int py, int t)
{
    int tx = 0, ty = 0, n = -1;
    const bool chroma = t >= 19;
    if (t < 16) n = nbr(P, r, 16, 16, -1, t, px, py, tx, ty);
    else if (t == 16) n = nbr(P, r, 16, 16, 0, -1, px, py, tx, ty);
    else if (t == 17) n = nbr(P, r, 16, 16, 16, -1, px, py, tx, ty);
    else if (t == 18) n = nbr(P, r, 16, 16, -1, -1, px, py, tx, ty);
    else if (t < 27) n = nbr(P, r, 8, 8, -1, t - 19, px, py, tx, ty);
    else if (t == 27) n = nbr(P, r, 8, 8, 0, -1, px, py, tx, ty);
    else if (t == 28) n = nbr(P, r, 8, 8, -1, -1, px, py, tx, ty);
    else return;
    const uint8_t av = (uint8_t)((n >= 0 ? 1 : 0) | (intra_ok(P, n) ? 2 : 0));
    const int16_t pos = (int16_t)(chroma ? (ty + 2) * TCW + tx + 1 : (ty + 2) * TYW + tx + 1);
    NbTab& T = L.nb;
    if (t < 16) { T.lpos[t] = pos; T.lav[t] = av; }
    else if (t == 16) { T.tpos = pos; T.tav = av; }
    else if (t == 17) { T.trpos = pos; T.trav = av; }
    else if (t == 18) { T.tlpos = pos; T.tlav = av; }
    else if (t < 27) { T.clpos[t - 19] = pos; T.clav[t - 19] = av; }
    else if (t == 27) { T.ctpos = pos; T.ctav = av; }
    else { T.ctlpos = pos; T.ctlav = av; }
}

// gather_nxn from the table: the block's samples inside the MB are the MB's own (always
// available, get_neighbour returns the MB itself), outside it the table's
DEV void gather_tab(IntraLds& L, bool fq, int bb, int N, int xO, int yO, int px, int py, bool cip, Nbr& n)
{
    const NbTab& T = L.nb;
    const int sh = cip ? 2 : 1;                                   // the availability bit to test
    auto own = [&](int x, int y) -> int {                         // tile index of own sample (x, y)
        return ((fq ? bb + 2 * y : bb * 16 + y) + 2) * TYW + x + 1;
    };
    // A: rows yO .. yO + N - 1 at column xO - 1 (CIP: every row's MB; else the first row's)
    int av0;
    if (xO > 0) av0 = 1;
    else if (cip) { av0 = 1; for (int i = 0; i < N; ++i) av0 &= (T.lav[yO + i] >> 1) & 1; }
    else av0 = T.lav[yO] & 1;
    // B, C, D
    int av1, av2, av3, bpos, cpos = 0, dpos;
    if (yO > 0) { av1 = 1; bpos = own(xO, yO - 1); }
    else { av1 = (T.tav & sh) != 0; bpos = T.tpos + xO; }
    if (xO + N < 16) {
        av2 = yO > 0 ? 1 : (T.tav & sh) != 0;
        cpos = yO > 0 ? own(xO + N, yO - 1) : T.tpos + xO + N;
    } else if (yO == 0) { av2 = (T.trav & sh) != 0; cpos = T.trpos + (xO + N - 16); }
    else av2 = 0;                                                // the MB to the right: later
    if (N == 4 && xO == 4 && (yO == 4 || yO == 12)) av2 = 0;     // :154
    if (N == 8 && xO == 8 && yO == 8) av2 = 0;                   // :376
    if (xO > 0 && yO > 0) { av3 = 1; dpos = own(xO - 1, yO - 1); }
    else if (xO > 0) { av3 = (T.tav & sh) != 0; dpos = T.tpos + xO - 1; }
    else if (yO > 0) { av3 = (T.lav[yO - 1] & sh) != 0; dpos = T.lpos[yO - 1]; }
    else { av3 = (T.tlav & sh) != 0; dpos = T.tlpos; }
    n.av[0] = av0; n.av[1] = av1; n.av[2] = av2; n.av[3] = av3;
    n.s[0] = av3 ? L.ty[dpos] : 0;
    for (int y = 0; y < N; ++y) n.s[17 + y] = av0 ? L.ty[xO > 0 ? own(xO - 1, yO + y) : T.lpos[yO + y]] : 0;
    for (int x = 0; x < N; ++x) n.s[1 + x] = av1 ? L.ty[bpos + x] : 0;
    for (int x = N; x < 2 * N; ++x) n.s[1 + x] = av1 ? (av2 ? L.ty[cpos + x - N] : n.s[N]) : 0;
    n.av[2] = av1;
}

// Intra16x16 from the table (intra_prediction.cc:624-735)
DEV int pred_16x16_tab(IntraLds& L, bool cip, int mode, int x, int y)
{
    const NbTab& T = L.nb;
    int a0 = T.lav[0] & 1, a1 = (T.tav >> (cip ? 1 : 0)) & 1;
    if (cip) { a0 = 1; for (int i = 0; i < 16; ++i) a0 &= (T.lav[i] >> 1) & 1; }
#define LT(k) L.ty[T.lpos[k]]
#define TP(k) L.ty[T.tpos + (k)]
    switch (mode) {
    case 0: return TP(x);
    case 1: return LT(y);
    case 2: {
        if (!a0 && !a1) return 128;
        int sum = 0;
        if (a0) for (int k = 0; k < 16; ++k) sum += LT(k);
        if (a1) for (int k = 0; k < 16; ++k) sum += TP(k);
        return (sum + (a0 ? 8 : 0) + (a1 ? 8 : 0)) >> (3 + a0 + a1);
    }
    default: {
        const int pd = L.ty[T.tlpos];
        int H = 0, V = 0;
        for (int k = 0; k < 8; ++k) {
            H += (k + 1) * (TP(8 + k) - (6 - k >= 0 ? TP(6 - k) : pd));
            V += (k + 1) * (LT(8 + k) - (6 - k >= 0 ? LT(6 - k) : pd));
        }
        const int a = 16 * (LT(15) + TP(15));
        const int b = (5 * H + 32) >> 6, c = (5 * V + 32) >> 6;
        return clip255((a + b * (x - 7) + c * (y - 7) + 16) >> 5);
    }
    }
#undef LT
#undef TP
}

// Chroma from the table (intra_prediction.cc:745-894), 4:2:0
DEV int pred_chroma_tab(IntraLds& L, bool cip, int mode, int pl, int x, int y)
{
    const NbTab& T = L.nb;
    int av0, av1, av2;
    if (cip) {
        av0 = 1; av2 = 1;
        for (int i = 0; i < 4; ++i) { av0 &= (T.clav[i] >> 1) & 1; av2 &= (T.clav[4 + i] >> 1) & 1; }
        av1 = (T.ctav >> 1) & 1;
    } else { av0 = T.clav[0] & 1; av2 = av0; av1 = T.ctav & 1; }
    const uint8_t* tc = L.tc[pl];
#define CL(k) tc[T.clpos[k]]
#define CT(k) tc[T.ctpos + (k)]
    switch (mode) {
    case 0: {
        const int xO = x & 4, yO = y & 4;
        int aA, aB;
        if ((xO == 0 && yO == 0) || (xO > 0 && yO > 0)) { aA = yO > 0 ? av2 : av0; aB = av1; }
        else if (xO > 0 && yO == 0) { aA = av1 ? 0 : av0; aB = av1; }
        else { aA = av2; aB = av2 ? 0 : av1; }
        if (!aA && !aB) return 128;
        int sum = 0;
        if (aA) for (int k = 0; k < 4; ++k) sum += CL(k + yO);
        if (aB) for (int k = 0; k < 4; ++k) sum += CT(k + xO);
        return (sum + (aA ? 2 : 0) + (aB ? 2 : 0)) >> (1 + aA + aB);
    }
    case 1: return CL(y);
    case 2: return CT(x);
    default: {
        const int pd = tc[T.ctlpos];
        int H = 0, V = 0;
        for (int k = 0; k < 4; ++k) {
            H += (k + 1) * (CT(4 + k) - (2 - k >= 0 ? CT(2 - k) : pd));
            V += (k + 1) * (CL(4 + k) - (2 - k >= 0 ? CL(2 - k) : pd));
        }
        const int a = 16 * (CL(7) + CT(7));
        const int b = (34 * H + 32) >> 6, c = (34 * V + 32) >> 6;
        return clip255((a + b * (x - 3) + c * (y - 3) + 16) >> 5);
    }
    }
#undef CL
#undef CT
}


// ------------------------------------------------------------------ loop filter
constexpr int DYW = 20, DYH = 40;      // luma tile: rows -8 .. 31, columns -4 .. 15 of the pair
constexpr int DCW = 12, DCH = 24;      // chroma tile: rows -8 .. 15, columns -4 .. 7
struct DbLds {
    uint8_t ty[DYH * DYW];
    uint8_t tc[2][DCH * DCW];
    uint8_t sv[2][4][16], sh[2][4][16], sh4[2][16];      // strength_ver / strength_hor / strength_hor[4]
    uint8_t fv[2][2][4], fh[2][2][4], fh4[2][2];          // filterVerEdgeFlag / filterHorEdgeFlag [chroma][edge]
};

DEV bool is_special(const MPic& P, int n)
{
    const int st = P.sl[P.mbs[n].slice].slice_type;
    return st == H264R_SLICE_SP || st == H264R_SLICE_SI;
}
DEV bool mb_intra(const MPic& P, int n) { return (P.mbs[n].flags & H264R_MBF_INTRA) != 0; }

// pic_motion_params of a 4x4 block (storage rows): the reference picture's identity -- the DPB
// slot, or for a field MB slot | 0x80 (| H264R_REF_BOTTOM for the bottom field): get_ref_pic's
// field pictures are never the frame (interpret_mb.cc:617-620, dpb.cc:1046-1055)
struct MvInfo { int ref[2], mx[2], my[2]; };
DEV MvInfo mvinfo(const MPic& P, int bx4, int by4)
{
    const int addr = (by4 >> 2) * P.wmb + (bx4 >> 2);
    const h264r_mb m = P.mbs[addr];
    const h264r_slice& sl = P.sl[m.slice];
    const bool fmb = (m.flags & H264R_MBF_FIELD) != 0;
    const int mbot = (addr / P.wmb) & 1, idx = by4 * P.W4 + bx4;
    MvInfo v;
    for (int l = 0; l < 2; ++l) {
        const int r = P.ref[l * P.mplane + idx];
        const uint32_t w = P.mv[l * P.mplane + idx];
        v.ref[l] = r < 0 ? -1 : !fmb ? sl.ref_slot[l][r] : (sl.ref_slot[l][r >> 1] | 0x80 | (((r & 1) != mbot) ? H264R_REF_BOTTOM : 0));
        v.mx[l] = (int16_t)(w & 0xFFFF);
        v.my[l] = (int16_t)(w >> 16);
    }
    return v;
}
DEV int cmp_mv(const MvInfo& a, int la, const MvInfo& b, int lb, int ml)               // deblock.cc:35-38
{
    return (int)(iabs(a.mx[la] - b.mx[lb]) >= 4) | (int)(iabs(a.my[la] - b.my[lb]) >= ml);
}
DEV int bs_mvs(const MvInfo& p, const MvInfo& q, int ml)                                 // deblock.cc:40-75
{
    const int p0 = p.ref[0], q0 = q.ref[0], p1 = p.ref[1], q1 = q.ref[1];
    if ((p0 == q0 && p1 == q1) || (p0 == q1 && p1 == q0)) {
        if (p0 != p1) {
            if (p0 == q0) return cmp_mv(p, 0, q, 0, ml) | cmp_mv(p, 1, q, 1, ml);
            return cmp_mv(p, 0, q, 1, ml) | cmp_mv(p, 1, q, 0, ml);
        }
        return (cmp_mv(p, 0, q, 0, ml) | cmp_mv(p, 1, q, 1, ml)) & (cmp_mv(p, 0, q, 1, ml) | cmp_mv(p, 1, q, 0, ml));
    }
    return 1;
}

// strength_vertical (deblock.cc:78-155) of row y of edge e of MB r
DEV int bs_ver(const MPic& P, int r, int e, int y)
{
    const h264r_mb q = P.mbs[r];
    const bool fq = (q.flags & H264R_MBF_FIELD) != 0;
    const int ml = fq ? 2 : 4, dy = 1 + fq;
    int xq, yq, lyp;
    mloc(P, r, 16, 16, e * 4, 0, xq, yq);
    const int P0 = mmb_at(P, 16, 16, xq - 1, yq, nullptr);
    const bool mixed = fq != is_fld(P, P0), special = is_special(P, P0) || is_special(P, r);
    if (e == 0 && special) return 4;
    if (!mixed && special) return 3;
    if (e > 0 && P.sl[q.slice].slice_type == H264R_SLICE_P && q.mb_type == H264R_P_SKIP) return 0;
    const int Pn = mmb_at(P, 16, 16, xq - 1, yq + dy * y, &lyp);
    const bool intra = mb_intra(P, Pn) || mb_intra(P, r);
    const int blkP = (lyp & 12) + ((xq - 1) & 15) / 4, blkQ = (y & 12) + e;
    if (e == 0 && intra) return 4;
    if (!mixed && intra) return 3;
    if (((q.cbp_blks >> blkQ) & 1) || ((P.mbs[Pn].cbp_blks >> blkP) & 1)) return 2;
    if (mixed) return 1;
    if (e > 0 && (q.mb_type == H264R_P_16x16 || q.mb_type == H264R_P_16x8)) return 0;
    const MvInfo mq = mvinfo(P, xq >> 2, (r / P.wmb) * 4 + (y >> 2));
    const MvInfo mp = mvinfo(P, (xq - 1) >> 2, (Pn / P.wmb) * 4 + (lyp >> 2));
    return bs_mvs(mq, mp, ml);
}

// strength_horizontal (deblock.cc:157-228) of columns 4 x4 .. 4 x4 + 3 of edge e (4: the second
// field edge) of MB r; f4 = filterHorEdgeFlag[0][4]
DEV int bs_hor(const MPic& P, int r, int e, int x4, bool f4)
{
    const h264r_mb q = P.mbs[r];
    const bool fq = (q.flags & H264R_MBF_FIELD) != 0;
    const int ml = fq ? 2 : 4, dy = 1 + (fq || ((e == 0 || e == 4) && f4));
    int xq, yq, lyq, lyp;
    mloc(P, r, 16, 16, 0, 0, xq, yq);
    yq += e == 4 ? 1 : dy * e * 4;
    const int Qn = mmb_at(P, 16, 16, xq, yq, &lyq), Pn = mmb_at(P, 16, 16, xq, yq - dy, &lyp);
    const bool mixed = fq != is_fld(P, Pn), special = is_special(P, Pn) || is_special(P, r);
    const bool field = is_fld(P, Pn) || fq, intra = mb_intra(P, Pn) || mb_intra(P, r);
    if (e == 0 && !field && (special || intra)) return 4;
    if (special || intra) return 3;
    if (e > 0 && e < 4 && P.sl[q.slice].slice_type == H264R_SLICE_P && q.mb_type == H264R_P_SKIP) return 0;
    if (((q.cbp_blks >> ((lyq & 12) + x4)) & 1) || ((P.mbs[Pn].cbp_blks >> ((lyp & 12) + x4)) & 1)) return 2;
    if (mixed) return 1;
    if (e > 0 && e < 4 && (q.mb_type == H264R_P_16x16 || q.mb_type == H264R_P_8x16)) return 0;
    const MvInfo mq = mvinfo(P, (xq >> 2) + x4, (Qn / P.wmb) * 4 + (lyq >> 2));
    const MvInfo mp = mvinfo(P, (xq >> 2) + x4, (Pn / P.wmb) * 4 + (lyp >> 2));
    return bs_mvs(mq, mp, ml);
}

// Deblock::strength's edge flags (deblock.cc:230-278) of MB r: bit 0..3 ver luma, 4..7 hor luma,
// the chroma edges 0 / 1 (4:2:0) follow the luma ones, bit 8 filterHorEdgeFlag[.][4]
DEV void edge_flags(const MPic& P, int r, DbLds& D, int h)
{
    const h264r_mb q = P.mbs[r];
    const int idc = P.sl[q.slice].deblock_idc;
    for (int c = 0; c < 2; ++c) {
        for (int e = 0; e < 4; ++e) D.fv[h][c][e] = D.fh[h][c][e] = 0;
        D.fh4[h][c] = 0;
    }
    if (idc == 1) return;
    const bool fq = (q.flags & H264R_MBF_FIELD) != 0;
    int xq, yq;
    mloc(P, r, 16, 16, 0, 0, xq, yq);
    const int Ln = mmb_at(P, 16, 16, xq - 1, yq, nullptr), Un = mmb_at(P, 16, 16, xq, yq - 1 - fq, nullptr);
    bool fl = false, ft = false;
    if (idc == 0) { fl = Ln >= 0; ft = Un >= 0; }
    else if (idc == 2) { fl = Ln >= 0 && P.mbs[Ln].slice == q.slice; ft = Un >= 0 && P.mbs[Un].slice == q.slice; }
    for (int c = 0; c < 2; ++c) {
        D.fv[h][c][0] = fl; D.fh[h][c][0] = ft;
        for (int e = 1; e < 4; ++e) D.fv[h][c][e] = D.fh[h][c][e] = 1;
        D.fh4[h][c] = ft && !fq && is_fld(P, Un);
    }
    if (q.flags & H264R_MBF_T8x8) D.fv[h][0][1] = D.fv[h][0][3] = D.fh[h][0][1] = D.fh[h][0][3] = 0;
    D.fv[h][1][2] = D.fv[h][1][3] = D.fh[h][1][2] = D.fh[h][1][3] = 0;
}

// filter_strong / filter_normal (deblock.cc:327-415) across the edge at q with step inc
DEV void filter_line(uint8_t* q, int inc, int alpha, int beta, int bS, bool chroma, int tc0)
{
#define Pp(i) q[-((i) + 1) * inc]
#define Qq(i) q[(i) * inc]
    const int p0 = Pp(0), p1 = Pp(1), p2 = Pp(2), q0 = Qq(0), q1 = Qq(1), q2 = Qq(2);
    if (!(iabs(p0 - q0) < alpha && iabs(p1 - p0) < beta && iabs(q1 - q0) < beta)) return;
    const int ap = iabs(p2 - p0), aq = iabs(q2 - q0);
    if (bS == 4) {
        int np0, np1, np2, nq0, nq1, nq2;
        if (!chroma && ap < beta && iabs(p0 - q0) < (alpha >> 2) + 2) {
            const int p3 = Pp(3);
            np0 = (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3;
            np1 = (p2 + p1 + p0 + q0 + 2) >> 2;
            np2 = (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3;
        } else { np0 = (2 * p1 + p0 + q1 + 2) >> 2; np1 = p1; np2 = p2; }
        if (!chroma && aq < beta && iabs(p0 - q0) < (alpha >> 2) + 2) {
            const int q3 = Qq(3);
            nq0 = (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3;
            nq1 = (p0 + q0 + q1 + q2 + 2) >> 2;
            nq2 = (2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3;
        } else { nq0 = (2 * q1 + q0 + p1 + 2) >> 2; nq1 = q1; nq2 = q2; }
        Pp(0) = (uint8_t)np0; Pp(1) = (uint8_t)np1; Pp(2) = (uint8_t)np2;
        Qq(0) = (uint8_t)nq0; Qq(1) = (uint8_t)nq1; Qq(2) = (uint8_t)nq2;
    } else {
        const int tc = chroma ? tc0 + 1 : tc0 + (ap < beta) + (aq < beta);
        const int delta = clip3(-tc, tc, (((q0 - p0) * 4) + (p1 - q1) + 4) >> 3);
        int np1 = p1, nq1 = q1;
        if (!chroma && ap < beta) np1 = p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 * 2)) >> 1);
        if (!chroma && aq < beta) nq1 = q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 * 2)) >> 1);
        Pp(0) = (uint8_t)clip255(p0 + delta);
        Qq(0) = (uint8_t)clip255(q0 - delta);
        Pp(1) = (uint8_t)np1; Qq(1) = (uint8_t)nq1;
    }
#undef Pp
#undef Qq
}

__constant__ uint8_t ALPHA[52] = {                                     // deblock.cc:294-299
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 4, 4, 5, 6, 7, 8, 9, 10, 12, 13,
    15, 17, 20, 22, 25, 28, 32, 36, 40, 45, 50, 56, 63, 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
__constant__ uint8_t BETA[52] = {                                      // deblock.cc:301-306
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4,
    6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18};
__constant__ uint8_t TC0[52][3] = {                                    // deblock.cc:310-324
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
    {0, 0, 0}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 1, 1}, {0, 1, 1}, {1, 1, 1},
    {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 2, 3},
    {1, 2, 3}, {2, 2, 3}, {2, 2, 4}, {2, 3, 4}, {2, 3, 4}, {3, 3, 5}, {3, 4, 6}, {3, 4, 6},
    {4, 5, 7}, {4, 5, 8}, {4, 6, 9}, {5, 7, 10}, {6, 8, 11}, {6, 8, 13}, {7, 10, 14}, {8, 11, 16},
    {9, 12, 18}, {10, 13, 20}, {11, 15, 23}, {13, 17, 25}};

// one line of filter_edge (deblock.cc:418-486) on the pair tile: MB r (half h of the pair), `edge`
// the sample offset or 1 (the second field edge, strength_hor[4]), line `pel`
DEV void filter_pel(const MPic& P, DbLds& D, int r, int h, bool chroma, int pl, bool vertical, bool fmode, int edge,
                    int pel, int px, int py)
{
    const h264r_mb q = P.mbs[r];
    const h264r_slice& sl = P.sl[q.slice];
    const uint8_t* St = vertical ? D.sv[h][chroma ? edge * 4 / 8 : edge / 4]
                      : edge == 1 ? D.sh4[h] : D.sh[h][chroma ? edge * 4 / 8 : edge / 4];
    const int nE = chroma ? 8 : 16, dy = 1 + fmode;
    int xI, yI;
    mloc(P, r, 16, 16, 0, 0, xI, yI);
    const int xP = chroma ? xI / 2 : xI, yP = chroma ? (yI + 1) / 2 : yI;
    int xJ = xI, yJ = yI;
    if (vertical) xJ += (edge - 1) * (chroma ? 2 : 1);
    else yJ += dy * (edge - 1) * (chroma ? 2 : 1) - (edge % 2);
    int Pn = mmb_at(P, 16, 16, xJ, yJ, nullptr);
    const bool mixed = vertical && !is_fld(P, r) && is_fld(P, Pn);
    const int bS = St[nE == 8 ? (pel << 1) + (mixed && (pel & 1)) : pel];
    if (!bS) return;
    if (vertical) Pn = mmb_at(P, 16, 16, xJ, yI + dy * pel * (chroma ? 2 : 1) + (chroma && mixed && (pel & 1)), nullptr);
    const h264r_mb pm = P.mbs[Pn];
    const int qPp = chroma ? pm.qp_c[pl - 1] : pm.qp_y, qPq = chroma ? q.qp_c[pl - 1] : q.qp_y;
    const int qPav = (qPp + qPq + 1) >> 1;
    const int iA = clip3(0, 51, qPav + sl.filter_offset_a), iB = clip3(0, 51, qPav + sl.filter_offset_b);
    const int gx = vertical ? xP + edge : xP + pel, gy = vertical ? yP + pel * dy : yP + dy * edge - (edge % 2);
    uint8_t* qptr;
    int pitch;
    if (!chroma) { qptr = &D.ty[(gy - py * 32 + 8) * DYW + gx - px * 16 + 4]; pitch = DYW; }
    else { qptr = &D.tc[pl - 1][(gy - py * 16 + 8) * DCW + gx - px * 8 + 4]; pitch = DCW; }
    filter_line(qptr, vertical ? 1 : dy * pitch, ALPHA[iA], BETA[iB], bS, chroma, bS < 4 ? TC0[iA][bS - 1] : 0);
}

}  // namespace
}  // namespace h264r

using namespace h264r;

// ------------------------------------------------------------------ kernels
// I_PCM and inter MBs, one 256-thread workgroup per MB: thread t is luma sample (t % 16, t / 16)
// and, for t < 128, chroma sample (t % 8, (t / 8) % 8) of plane 1 + t / 64.
extern "C" __global__ __launch_bounds__(256) void k_mbaff_inter(h264r_batch b, int* err)
{
    __shared__ ResLds R;
    const int nmb = b.width_mbs * b.height_mbs, pic = blockIdx.x / nmb, r = blockIdx.x % nmb, t = threadIdx.x;
    const MPic P = mpic(b, pic);
    const h264r_mb m = P.mbs[r];
    const bool pcm = m.mb_type == H264R_I_PCM;
    if ((m.flags & H264R_MBF_INTRA) && !pcm) return;
    const int Wl = P.wmb * 16, Wc = P.wmb * 8;
    const int16_t* lv = b.levels + m.coef_off;
    int gx, gy;
    if (pcm) {                                                             // mb_pred_ipcm decoder.cc:149-168
        const uint8_t* raw = reinterpret_cast<const uint8_t*>(lv);
        mloc(P, r, 16, 16, t & 15, t >> 4, gx, gy);
        P.out[0][(size_t)gy * Wl + gx] = raw[t];
        if (t < 128) {
            const int pl = 1 + (t >> 6), k = t & 63;
            mloc(P, r, 8, 8, k & 7, k >> 3, gx, gy);
            P.out[pl][(size_t)gy * Wc + gx] = raw[256 + (pl - 1) * 64 + k];
        }
        return;
    }
    mb_residual(m, lv, *P.q, R, t);
    {
        const int x = t & 15, y = t >> 4;
        const int v = clip255(R.cof[0][t] + inter_sample(P, r, 0, x, y, err));
        mloc(P, r, 16, 16, x, y, gx, gy);
        P.out[0][(size_t)gy * Wl + gx] = (uint8_t)v;
    }
    if (t < 128) {
        const int pl = 1 + (t >> 6), k = t & 63, x = k & 7, y = k >> 3;
        const int v = clip255(R.cof[pl][k] + inter_sample(P, r, pl, x, y, err));
        mloc(P, r, 8, 8, x, y, gx, gy);
        P.out[pl][(size_t)gy * Wc + gx] = (uint8_t)v;
    }
}

// Intra MBs of the pairs on anti-diagonal `diag` (x + 2 y), one 256-thread workgroup per pair.
extern "C" __global__ __launch_bounds__(256) void k_mbaff_intra(h264r_batch b, int diag, int* err)
{
    __shared__ IntraLds L;
    const int HP = b.height_mbs / 2, pic = blockIdx.x / HP, py = blockIdx.x % HP, px = diag - 2 * py, t = threadIdx.x;
    if (px < 0 || px >= b.width_mbs) return;
    const MPic P = mpic(b, pic);
    const int rt = (2 * py) * P.wmb + px, rb = rt + P.wmb;
    const bool it = (P.mbs[rt].flags & H264R_MBF_INTRA) && P.mbs[rt].mb_type != H264R_I_PCM;
    const bool ib = (P.mbs[rb].flags & H264R_MBF_INTRA) && P.mbs[rb].mb_type != H264R_I_PCM;
    if (!it && !ib) return;
    const int Wl = P.wmb * 16, Hl = P.hmb * 16, Wc = P.wmb * 8, Hc = P.hmb * 8;
    for (int k = t; k < TYH * TYW; k += 256) {
        const int x = k % TYW - 1, y = k / TYW - 2, gx = px * 16 + x, gy = py * 32 + y;
        L.ty[k] = (gx >= 0 && gx < Wl && gy >= 0 && gy < Hl) ? P.out[0][(size_t)gy * Wl + gx] : 0;
    }
    for (int k = t; k < 2 * TCH * TCW; k += 256) {
        const int pl = k / (TCH * TCW), e = k % (TCH * TCW), x = e % TCW - 1, y = e / TCW - 2;
        const int gx = px * 8 + x, gy = py * 16 + y;
        L.tc[pl][e] = (gx >= 0 && gx < Wc && gy >= 0 && gy < Hc) ? P.out[1 + pl][(size_t)gy * Wc + gx] : 0;
    }
    __syncthreads();
    for (int half = 0; half < 2; ++half) {
        const int r = half ? rb : rt;
        if (!(half ? ib : it)) continue;
        const h264r_mb m = P.mbs[r];
        nb_table(P, L, r, px, py, t);                                  // ordered by mb_residual's barriers
        mb_residual(m, b.levels + m.coef_off, *P.q, L.R, t);
        const bool fq = (m.flags & H264R_MBF_FIELD) != 0, cip = P.cip != 0;
        int gx, gy;
        if (m.mb_type == H264R_I_16x16) {
            const int x = t & 15, y = t >> 4;
            const int v = clip255(L.R.cof[0][t] + pred_16x16_tab(L, cip, m.i16_mode, x, y));
            __syncthreads();                                           // every prediction reads the old tile
            mloc(P, r, 16, 16, x, y, gx, gy);
            TY(L, gx - px * 16, gy - py * 32) = (uint8_t)v;
        } else {
            const int N = m.mb_type == H264R_I_4x4 ? 4 : 8, nblk = N == 4 ? 16 : 4;
            for (int bk = 0; bk < nblk; ++bk) {
                const int xO = N == 4 ? ((bk >> 2) & 1) * 8 + (bk & 1) * 4 : (bk & 1) * 8;
                const int yO = N == 4 ? (bk >> 3) * 8 + ((bk >> 1) & 1) * 4 : (bk >> 1) * 8;
                if (t < N * N) {
                    Nbr n, f;
                    gather_tab(L, fq, half, N, xO, yO, px, py, cip, n);
                    if (N == 8) filter_8x8(n, f); else f = n;
                    const int mode = (m.ipred[bk >> 1] >> ((bk & 1) * 4)) & 15;
                    const int x = t % N, y = t / N;
                    const int v = clip255(L.R.cof[0][(yO + y) * 16 + xO + x] + pred_nxn(f, N, mode, x, y));
                    mloc(P, r, 16, 16, xO + x, yO + y, gx, gy);
                    TY(L, gx - px * 16, gy - py * 32) = (uint8_t)v;
                }
                __syncthreads();
            }
        }
        int v = 0, cx = 0, cy = 0, pl = 0;
        if (t < 128) {
            pl = t >> 6; cx = t & 7; cy = (t >> 3) & 7;
            v = clip255(L.R.cof[1 + pl][cy * 8 + cx] + pred_chroma_tab(L, cip, m.chroma_mode, pl, cx, cy));
        }
        __syncthreads();
        if (t < 128) {
            mloc(P, r, 8, 8, cx, cy, gx, gy);
            TC(L, pl, gx - px * 8, gy - py * 16) = (uint8_t)v;
        }
        __syncthreads();
    }
    for (int k = t; k < 32 * 16; k += 256) {
        const int x = k & 15, y = k >> 4;
        P.out[0][(size_t)(py * 32 + y) * Wl + px * 16 + x] = TY(L, x, y);
    }
    for (int k = t; k < 2 * 16 * 8; k += 256) {
        const int pl = k >> 7, e = k & 127, x = e & 7, y = e >> 3;
        P.out[1 + pl][(size_t)(py * 16 + y) * Wc + px * 8 + x] = TC(L, pl, x, y);
    }
    (void)err;
}

// The loop filter of the pairs on anti-diagonal `diag`, one wave per pair: the strengths of both
// MBs, then each MB's vertical and horizontal edges in the reference's order (deblock.cc:488-552);
// lanes 0..15 the luma lines of an edge, 16..23 Cb, 24..31 Cr.
extern "C" __global__ __launch_bounds__(64) void k_mbaff_deblock(h264r_batch b, int diag, int* err)
{
    __shared__ DbLds D;
    const int HP = b.height_mbs / 2, pic = blockIdx.x / HP, py = blockIdx.x % HP, px = diag - 2 * py, t = threadIdx.x;
    if (px < 0 || px >= b.width_mbs) return;
    const MPic P = mpic(b, pic);
    const int r0 = (2 * py) * P.wmb + px;
    const int Wl = P.wmb * 16, Hl = P.hmb * 16, Wc = P.wmb * 8, Hc = P.hmb * 8;
    if (t < 2) edge_flags(P, r0 + t * P.wmb, D, t);
    for (int k = t; k < DYH * DYW; k += 64) {
        const int gx = px * 16 + k % DYW - 4, gy = py * 32 + k / DYW - 8;
        D.ty[k] = (gx >= 0 && gx < Wl && gy >= 0 && gy < Hl) ? P.out[0][(size_t)gy * Wl + gx] : 0;
    }
    for (int k = t; k < 2 * DCH * DCW; k += 64) {
        const int pl = k / (DCH * DCW), e = k % (DCH * DCW);
        const int gx = px * 8 + e % DCW - 4, gy = py * 16 + e / DCW - 8;
        D.tc[pl][e] = (gx >= 0 && gx < Wc && gy >= 0 && gy < Hc) ? P.out[1 + pl][(size_t)gy * Wc + gx] : 0;
    }
    __syncthreads();
    for (int h = 0; h < 2; ++h) {                                     // Deblock::strength
        const int r = r0 + h * P.wmb;
        for (int e = 0; e < 4; ++e) {
            if (t < 16 && D.fv[h][0][e]) D.sv[h][e][t] = (uint8_t)bs_ver(P, r, e, t);
            if (t >= 16 && t < 20 && D.fh[h][0][e]) {
                const int v = bs_hor(P, r, e, t - 16, D.fh4[h][0]);
                for (int k = 0; k < 4; ++k) D.sh[h][e][(t - 16) * 4 + k] = (uint8_t)v;
            }
        }
        if (t >= 20 && t < 24 && D.fh4[h][0]) {
            const int v = bs_hor(P, r, 4, t - 20, true);
            for (int k = 0; k < 4; ++k) D.sh4[h][(t - 20) * 4 + k] = (uint8_t)v;
        }
    }
    __syncthreads();
    const bool chroma = t >= 16 && t < 32;
    const int pl = t < 24 ? 1 : 2, pel = chroma ? (t - 16) & 7 : t;
    for (int h = 0; h < 2; ++h) {
        const int r = r0 + h * P.wmb;
        const bool fq = is_fld(P, r);
        for (int e = 0; e < 4; ++e) {                                  // filter_vertical
            if (t < 16 && D.fv[h][0][e]) filter_pel(P, D, r, h, false, 0, true, fq, e * 4, pel, px, py);
            if (chroma && D.fv[h][1][e]) filter_pel(P, D, r, h, true, pl, true, fq, e * 4, pel, px, py);
            __syncthreads();
        }
        for (int e = 0; e < 4; ++e) {                                  // filter_horizontal
            const bool split_l = e == 0 && D.fh4[h][0], split_c = e == 0 && D.fh4[h][1];
            if (t < 16 && D.fh[h][0][e]) filter_pel(P, D, r, h, false, 0, false, split_l || fq, 0 + e * 4, pel, px, py);
            if (chroma && D.fh[h][1][e]) filter_pel(P, D, r, h, true, pl, false, split_c || fq, e * 4, pel, px, py);
            __syncthreads();
            if (split_l || split_c) {
                if (t < 16 && split_l && D.fh[h][0][0]) filter_pel(P, D, r, h, false, 0, false, true, 1, pel, px, py);
                if (chroma && split_c && D.fh[h][1][0]) filter_pel(P, D, r, h, true, pl, false, true, 1, pel, px, py);
                __syncthreads();
            }
        }
    }
    for (int k = t; k < DYH * DYW; k += 64) {
        const int x = k % DYW - 4, y = k / DYW - 8, gx = px * 16 + x, gy = py * 32 + y;
        if ((x < 0 && y < 0) || gx < 0 || gy < 0 || gy >= Hl) continue;
        P.out[0][(size_t)gy * Wl + gx] = D.ty[k];
    }
    for (int k = t; k < 2 * DCH * DCW; k += 64) {
        const int pl2 = k / (DCH * DCW), e = k % (DCH * DCW), x = e % DCW - 4, y = e / DCW - 8;
        const int gx = px * 8 + x, gy = py * 16 + y;
        if ((x < 0 && y < 0) || gx < 0 || gy < 0 || gy >= Hc) continue;
        P.out[1 + pl2][(size_t)gy * Wc + gx] = D.tc[pl2][e];
    }
    (void)err;
}
