// mb_inter.h -- one inter (or I_PCM) macroblock per 64-lane wave, registers only.
//
//   Decoder::mb_pred_inter decoder.cc:212-262 (partition walk = per-4x4 motion),
//   InterPrediction::inter_pred / get_block_luma / get_block_chroma / mc_prediction /
//   bi_prediction inter_prediction.cc:53-536,
//   Transform::inverse_transform_inter transform.cc:1051-1095 (inverse_4x4 :597-641,
//   chroma DC :875-889, construction :913-984).
//
// Lane roles (fixed for the whole MB, so nothing goes through LDS):
//   luma   lane = 4x4 block (raster) * 4 + row          -> 4 samples of one row
//   chroma lane = plane << 5 | 4x4 block << 3 | half << 2 | row
//                                                       -> 2 samples (cols 2*half, +1)
// The luma 4x4 inverse transform runs rows in-lane and columns across the 4 lanes
// of a quad (DPP quad broadcasts); the chroma one exchanges half-rows with a lane
// swizzle and columns with quad broadcasts.  Every global load whose address does
// not depend on the MB record (motion) is issued before the record arrives, and the
// level / scale loads are issued before motion compensation starts.
#pragma once
#include "mb_recon.h"

namespace h264r {

template <int K>
DEV int quad_bcast(int v)       // value of lane K of this lane's quad
{
    return __builtin_amdgcn_update_dpp(0, v, K * 0x55, 0xF, 0xF, false);
}

// Column pass of inverse_4x4 (transform.cc:619-640) for the lane holding row r of
// the block: t[k] = row k's value in this column.  Returns ((o_r + 32) >> 6).
DEV int idct4_col_row(int t0, int t1, int t2, int t3, int r)
{
    const int e0 = t0 + t2, e1 = t0 - t2, e2 = (t1 >> 1) - t3, e3 = t1 + (t3 >> 1);
    const bool outer = r == 0 || r == 3;
    const int x = outer ? e0 : e1, y = outer ? e3 : e2;
    return ((r < 2 ? x + y : x - y) + 32) >> 6;
}

DEV uint2 ld8(const void* p) { return *reinterpret_cast<const uint2*>(p); }

// Inter MB or I_PCM `a` of picture `pic`.  `mot` is the picture's resolved motion
// ([list][H4][W4], k_prep); R is only used by 8x8-transform MBs.
DEV void inter_mb2(const h264r_batch& b, const Geom& g, int pic, int a, int lane, const uint2* __restrict__ mot,
                   ResLds& R)
{
    const int mbx = a % g.wmb, mby = a / g.wmb;
    // ---- motion of this lane's luma and chroma blocks: independent of the record
    const int bi = lane >> 2, r = lane & 3, bx = bi & 3, by = bi >> 2;
    const int cpl = lane >> 5, cb = (lane >> 3) & 3, chalf = (lane >> 2) & 1, crow = lane & 3;
    const int cbx = (cb & 1) * 2 + chalf, cby = (cb >> 1) * 2 + (crow >> 1);
    const int li = (mby * 4 + by) * g.W4 + mbx * 4 + bx, ci = (mby * 4 + cby) * g.W4 + mbx * 4 + cbx;
    const uint2 lm0 = mot[li], lm1 = mot[g.motion_plane + li];
    const uint2 cm0 = mot[ci], cm1 = mot[g.motion_plane + ci];

    const h264r_mb m = load_mb(&b.mbs[(size_t)pic * g.nmb + a]);
    const PicPtrs o = out_planes(b, g, pic);
    const int16_t* lv = b.levels + m.coef_off;
    if (m.mb_type == H264R_I_PCM) { pcm_mb(m, lv, g, o, mbx, mby, lane); return; }
    if (mb_is_intra(m)) return;

    // ---- residual inputs (levels + scales), issued before MC
    const int cbpl = m.cbp & 15, cbpc = m.cbp >> 4;
    const int t8 = (m.flags & H264R_MBF_T8x8) != 0;
    const h264r_quant* __restrict__ q = &b.quant[pic];
    uint2 llev = make_uint2(0, 0), lsc = make_uint2(0, 0);
    const int qpl = m.qp_scaled[0];
    const int loff = b8_offset(m.cbp, (by >> 1) * 2 + (bx >> 1));
    if (!t8 && loff >= 0) {
        llev = ld8(lv + loff + ((by & 1) * 2 + (bx & 1)) * 16 + r * 4);
        lsc = ld8(&q->scale4x4[1][0][qpl % 6][r * 4]);
    }
    const int qpc = m.qp_scaled[1 + cpl];
    uint32_t clev = 0, csc = 0;
    uint2 cdc = make_uint2(0, 0);
    int cdc_scale = 0;
    if (cbpc) {
        const LevelOffs lo = level_offsets(m);
        cdc = ld8(lv + lo.cdc + cpl * 4);
        cdc_scale = q->scale4x4[1][1 + cpl][qpc % 6][0];
        if (cbpc == 2) {
            clev = *reinterpret_cast<const uint32_t*>(lv + lo.cac + cpl * 64 + cb * 16 + crow * 4 + chalf * 2);
            csc = *reinterpret_cast<const uint32_t*>(&q->scale4x4[1][1 + cpl][qpc % 6][crow * 4 + chalf * 2]);
        }
    }

    // ---- prediction
    const h264r_slice* __restrict__ sl = &b.slices[(size_t)pic * b.slice_stride + m.slice];
    int predL[4];
    {
        const uint2 w[2] = {lm0, lm1};
        const int r0 = (int8_t)(lm0.y & 255), r1 = (int8_t)(lm1.y & 255);
        const int dir = (r0 >= 0 && r1 >= 0) ? 2 : (r0 >= 0 ? 0 : 1);
        int v[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
        for (int l = 0; l < 2; ++l) {
            const int rr = l ? r1 : r0;
            if (rr < 0) continue;
            const int slot = (int8_t)((w[l].y >> 8) & 255);
            const uint8_t* img = slot >= 0 && slot < H264R_MAX_SLOTS && rr < H264R_MAX_REFS ? b.ref_planes[slot * 3] : nullptr;
            if (!img) { v[l][0] = v[l][1] = v[l][2] = v[l][3] = 128; continue; }
            const int vx = (mbx * 4 + bx) * 16 + (int16_t)(w[l].x & 0xFFFF);
            const int vy = (mby * 4 + by) * 16 + (int16_t)(w[l].x >> 16);
#ifdef H264R_EXP_FULLPEL
            luma_pred4<0, 0>(img, g.W, g.H, vx >> 2, (vy >> 2) + r, 0, 0, v[l]);
#else
            luma_pred4(img, g.W, g.H, vx >> 2, (vy >> 2) + r, vx & 3, vy & 3, v[l]);
#endif
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) predL[c] = wp_combine(sl, dir, r0, r1, v[0][c], v[1][c], 0);
    }
    int predC[2];
    {
        const uint2 w[2] = {cm0, cm1};
        const int r0 = (int8_t)(cm0.y & 255), r1 = (int8_t)(cm1.y & 255);
        const int dir = (r0 >= 0 && r1 >= 0) ? 2 : (r0 >= 0 ? 0 : 1);
        int v[2][2] = {{0, 0}, {0, 0}};
#pragma unroll
        for (int l = 0; l < 2; ++l) {
            const int rr = l ? r1 : r0;
            if (rr < 0) continue;
            const int slot = (int8_t)((w[l].y >> 8) & 255);
            const uint8_t* img = slot >= 0 && slot < H264R_MAX_SLOTS && rr < H264R_MAX_REFS ? b.ref_planes[slot * 3 + 1 + cpl] : nullptr;
            if (!img) { v[l][0] = v[l][1] = 128; continue; }
            const int vx = (mbx * 4 + cbx) * 16 + (int16_t)(w[l].x & 0xFFFF);
            const int vy = (mby * 4 + cby) * 16 + (int16_t)(w[l].x >> 16);
            chroma_pred2(img, g.Wc, g.Hc, vx >> 3, (vy >> 3) + (crow & 1), vx & 7, vy & 7, v[l]);
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) predC[c] = wp_combine(sl, dir, r0, r1, v[0][c], v[1][c], 1 + cpl);
    }

    // ---- luma residual (transform.cc:1058-1073)
    int resL[4] = {0, 0, 0, 0};
#ifdef H264R_EXP_NORESID
    if (0) {
#else
    if (cbpl) {
#endif
        if (!t8) {
            const int per = qpl / 6;
            int d[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int lev = (int16_t)((c & 2 ? llev.y : llev.x) >> (16 * (c & 1)));
                const int sc = (int16_t)((c & 2 ? lsc.y : lsc.x) >> (16 * (c & 1)));
                d[c] = dq4(lev, sc, per);
            }
            int t[4];
            idct4(d[0], d[1], d[2], d[3], t[0], t[1], t[2], t[3]);      // row pass, in lane
#pragma unroll
            for (int c = 0; c < 4; ++c)                                  // column pass across the quad
                resL[c] = idct4_col_row(quad_bcast<0>(t[c]), quad_bcast<1>(t[c]), quad_bcast<2>(t[c]),
                                        quad_bcast<3>(t[c]), r);
        } else {
            residual_mb(m, lv, q, R, lane);                              // 8x8 transform: LDS path
#pragma unroll
            for (int c = 0; c < 4; ++c) resL[c] = R.lum[by * 4 + r][bx * 4 + c];
        }
    }
    // ---- chroma residual (transform.cc:1081-1091, DC :875-889)
    int resC[2] = {0, 0};
#ifdef H264R_EXP_NORESID
    if (0) {
#else
    if (cbpc) {
#endif
        const int per = qpc / 6;
        const int c00 = (int16_t)(cdc.x & 0xFFFF), c01 = (int16_t)(cdc.x >> 16);
        const int c10 = (int16_t)(cdc.y & 0xFFFF), c11 = (int16_t)(cdc.y >> 16);
        const int e00 = c00 + c01, e01 = c00 - c01, e10 = c10 + c11, e11 = c10 - c11;
        const int f = cb == 0 ? e00 + e10 : cb == 1 ? e01 + e11 : cb == 2 ? e00 - e10 : e01 - e11;
        const int dc = ((f * cdc_scale) * (1 << per)) >> 5;
        int k0 = 0, k1 = 0;                                           // my two coefficients
        if (cbpc == 2) {
            k0 = dq4((int16_t)(clev & 0xFFFF), (int16_t)(csc & 0xFFFF), per);
            k1 = dq4((int16_t)(clev >> 16), (int16_t)(csc >> 16), per);
        }
        if (crow == 0 && chalf == 0) k0 = dc;
        // row pass: the other half of my row sits in lane ^ 4
        const int o0 = __shfl_xor(k0, 4), o1 = __shfl_xor(k1, 4);
        const int d0 = chalf ? o0 : k0, d1 = chalf ? o1 : k1, d2 = chalf ? k0 : o0, d3 = chalf ? k1 : o1;
        int t[4];
        idct4(d0, d1, d2, d3, t[0], t[1], t[2], t[3]);
        const int u0 = chalf ? t[2] : t[0], u1 = chalf ? t[3] : t[1];
        resC[0] = idct4_col_row(quad_bcast<0>(u0), quad_bcast<1>(u0), quad_bcast<2>(u0), quad_bcast<3>(u0), crow);
        resC[1] = idct4_col_row(quad_bcast<0>(u1), quad_bcast<1>(u1), quad_bcast<2>(u1), quad_bcast<3>(u1), crow);
    }

    // ---- construction (transform.cc:913-984): rec = clip1(pred + rres)
    {
        uint32_t w = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) w |= (uint32_t)clip255(predL[c] + resL[c]) << (8 * c);
        *reinterpret_cast<uint32_t*>(o.y + (size_t)(mby * 16 + by * 4 + r) * g.W + mbx * 16 + bx * 4) = w;
    }
    {
        const uint32_t w = (uint32_t)clip255(predC[0] + resC[0]) | ((uint32_t)clip255(predC[1] + resC[1]) << 8);
        uint8_t* dst = cpl ? o.v : o.u;
        *reinterpret_cast<uint16_t*>(dst + (size_t)(mby * 8 + (cb >> 1) * 4 + crow) * g.Wc + mbx * 8 + (cb & 1) * 4 +
                                     chalf * 2) = (uint16_t)w;
    }
}

}  // namespace h264r
