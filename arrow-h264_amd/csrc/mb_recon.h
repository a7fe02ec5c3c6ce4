// mb_recon.h -- per-macroblock reconstruction as wave-level device functions
// (one 64-lane wave per MB, wave-synchronous LDS scratch), used by k_inter
// (fully parallel inter MBs) and k_picture (intra MBs along the wavefront).
//
//   residual_mb : dequant transform.cc:394-456, DC transforms :825-910,
//                 inverse_4x4 :597-641, inverse_8x8 :643-733
//   (inter MBs: mb_inter.h)
//   intra_mb    : Decoder::mb_pred_intra decoder.cc:170-208, IntraPrediction
//                 intra_prediction.cc:42-904, inverse_transform_{4x4,8x8,16x16,chroma}
//                 transform.cc:986-1049
#pragma once
#include "device_common.h"

namespace h264r {


// --------------------------------------------------------------------------------
// Residual of one MB into LDS (dequant transform.cc:394-456, DC transforms
// :825-910, inverse_4x4 :597-641, inverse_8x8 :643-733).  All 64 lanes take part.
//   lum[16][16], chr[2][8][8] receive the residual (mb_rres); both zeroed first.
// --------------------------------------------------------------------------------
struct ResLds {
    int lum[16][16];
    int chr[2][8][8];
};

DEV void residual_mb(const h264r_mb& m, const int16_t* __restrict__ lv, const h264r_quant* __restrict__ q,
                     ResLds& R, int lane)
{
    const int inter = mb_is_intra(m) ? 0 : 1;
    const int t8 = (m.flags & H264R_MBF_T8x8) != 0;
    const int i16 = m.mb_type == H264R_I_16x16;
    const int cbpc = m.cbp >> 4;
    const LevelOffs o = level_offsets(m);
    int* lum = &R.lum[0][0];
    int* chr = &R.chr[0][0][0];
    for (int k = lane; k < 256; k += 64) lum[k] = 0;
    for (int k = lane; k < 128; k += 64) chr[k] = 0;
    wave_sync();

    // ---- luma levels -> dequantised coefficients (cof)
    {
        const int qp = m.qp_scaled[0], per = qp / 6, rem = qp % 6;
        if (!t8) {
            int b = lane >> 2, r = lane & 3, bx = b & 3, by = b >> 2;
            int b8 = (by >> 1) * 2 + (bx >> 1), b4 = (by & 1) * 2 + (bx & 1);
            const int off = b8_offset(m.cbp, b8);
            if (off >= 0) {
                const int16_t* p = lv + off + b4 * 16 + r * 4;
                const int16_t* sc = &q->scale4x4[inter][0][rem][r * 4];
                for (int c = 0; c < 4; ++c) {
                    int pos = r * 4 + c;
                    if (i16 && pos == 0) continue;
                    int lev = p[c];
                    if (lev) R.lum[by * 4 + r][bx * 4 + c] = dq4(lev, sc[c], per);
                }
            }
        } else {
            int k = lane >> 4, row = (lane >> 1) & 7, half = lane & 1;
            const int off = b8_offset(m.cbp, k);
            if (off >= 0) {
                const int16_t* p = lv + off + row * 8 + half * 4;
                const int16_t* sc = &q->scale8x8[inter][0][rem][row * 8 + half * 4];
                for (int c = 0; c < 4; ++c) {
                    int lev = p[c];
                    if (lev) R.lum[(k >> 1) * 8 + row][(k & 1) * 8 + half * 4 + c] = dq8(lev, sc[c], per);
                }
            }
        }
    }
    // ---- chroma AC (positions 1..15 only)
    if (cbpc == 2 && lane < 32) {
        int pl = lane >> 4, blk = (lane >> 2) & 3, r = lane & 3;
        int qP = m.qp_scaled[1 + pl];
        const int16_t* p = lv + o.cac + pl * 64 + blk * 16 + r * 4;
        const int16_t* sc = &q->scale4x4[inter][1 + pl][qP % 6][r * 4];
        for (int c = 0; c < 4; ++c) {
            if (r == 0 && c == 0) continue;
            int lev = p[c];
            if (lev) R.chr[pl][(blk >> 1) * 4 + r][(blk & 1) * 4 + c] = dq4(lev, sc[c], qP / 6);
        }
    }
    // ---- chroma DC: 2x2 Hadamard + scale (transform_chroma_dc :875-889)
    if (cbpc && (lane == 32 || lane == 33)) {
        int pl = lane - 32, qP = m.qp_scaled[1 + pl];
        int scale = q->scale4x4[inter][1 + pl][qP % 6][0];
        const int16_t* p = lv + o.cdc + pl * 4;
        int c00 = p[0], c01 = p[1], c10 = p[2], c11 = p[3];
        int e00 = c00 + c01, e01 = c00 - c01, e10 = c10 + c11, e11 = c10 - c11;
        int f[4] = {e00 + e10, e01 + e11, e00 - e10, e01 - e11};
        for (int k = 0; k < 4; ++k)
            R.chr[pl][(k >> 1) * 4][(k & 1) * 4] = ((f[k] * scale) * (1 << (qP / 6))) >> 5;
    }
    // ---- luma DC of I_16x16: 4x4 Hadamard + scale (transform_luma_dc :825-856)
    if (i16 && lane == 48) {
        int qP = m.qp_scaled[0];
        int scale = q->scale4x4[0][0][qP % 6][0];
        const int16_t* p = lv + o.ldc;
        int e[4][4];
        for (int i = 0; i < 4; ++i) {
            int c0 = p[i * 4 + 0], c1 = p[i * 4 + 1], c2 = p[i * 4 + 2], c3 = p[i * 4 + 3];
            int d0 = c0 + c2, d1 = c0 - c2, d2 = c1 - c3, d3 = c1 + c3;
            e[i][0] = d0 + d3; e[i][1] = d1 + d2; e[i][2] = d1 - d2; e[i][3] = d0 - d3;
        }
        for (int j = 0; j < 4; ++j) {
            int h0 = e[0][j] + e[2][j], h1 = e[0][j] - e[2][j];
            int h2 = e[1][j] - e[3][j], h3 = e[1][j] + e[3][j];
            int f[4] = {h0 + h3, h1 + h2, h1 - h2, h0 - h3};
            for (int i = 0; i < 4; ++i) {
                int v = qP >= 36 ? (f[i] * scale) * (1 << (qP / 6 - 6))
                                 : (f[i] * scale + (1 << (5 - qP / 6))) >> (6 - qP / 6);
                R.lum[i * 4][j * 4] = v;
            }
        }
    }
    wave_sync();

    // ---- inverse transforms: rows
    if (!t8) {
        int b = lane >> 2, r = lane & 3, bx = b & 3, by = b >> 2;
        int* row = &R.lum[by * 4 + r][bx * 4];
        int o0, o1, o2, o3;
        idct4(row[0], row[1], row[2], row[3], o0, o1, o2, o3);
        row[0] = o0; row[1] = o1; row[2] = o2; row[3] = o3;
    } else if (lane < 32) {
        int k = lane >> 3, r = lane & 7;
        int* row = &R.lum[(k >> 1) * 8 + r][(k & 1) * 8];
        int in[8], out[8];
        for (int i = 0; i < 8; ++i) in[i] = row[i];
        idct8(in, out);
        for (int i = 0; i < 8; ++i) row[i] = out[i];
    }
    if (lane >= 32) {
        int l = lane - 32, pl = l >> 4, blk = (l >> 2) & 3, r = l & 3;
        int* row = &R.chr[pl][(blk >> 1) * 4 + r][(blk & 1) * 4];
        int o0, o1, o2, o3;
        idct4(row[0], row[1], row[2], row[3], o0, o1, o2, o3);
        row[0] = o0; row[1] = o1; row[2] = o2; row[3] = o3;
    }
    wave_sync();
    // ---- columns, final (x + 32) >> 6
    if (!t8) {
        int b = lane >> 2, c = lane & 3, bx = b & 3, by = b >> 2;
        int x = bx * 4 + c, y0 = by * 4;
        int o0, o1, o2, o3;
        idct4(R.lum[y0][x], R.lum[y0 + 1][x], R.lum[y0 + 2][x], R.lum[y0 + 3][x], o0, o1, o2, o3);
        R.lum[y0][x] = (o0 + 32) >> 6; R.lum[y0 + 1][x] = (o1 + 32) >> 6;
        R.lum[y0 + 2][x] = (o2 + 32) >> 6; R.lum[y0 + 3][x] = (o3 + 32) >> 6;
    } else if (lane < 32) {
        int k = lane >> 3, c = lane & 7;
        int x = (k & 1) * 8 + c, y0 = (k >> 1) * 8;
        int in[8], out[8];
        for (int i = 0; i < 8; ++i) in[i] = R.lum[y0 + i][x];
        idct8(in, out);
        for (int i = 0; i < 8; ++i) R.lum[y0 + i][x] = (out[i] + 32) >> 6;
    }
    if (lane >= 32) {
        int l = lane - 32, pl = l >> 4, blk = (l >> 2) & 3, c = l & 3;
        int x = (blk & 1) * 4 + c, y0 = (blk >> 1) * 4;
        int o0, o1, o2, o3;
        idct4(R.chr[pl][y0][x], R.chr[pl][y0 + 1][x], R.chr[pl][y0 + 2][x], R.chr[pl][y0 + 3][x], o0, o1, o2, o3);
        R.chr[pl][y0][x] = (o0 + 32) >> 6; R.chr[pl][y0 + 1][x] = (o1 + 32) >> 6;
        R.chr[pl][y0 + 2][x] = (o2 + 32) >> 6; R.chr[pl][y0 + 3][x] = (o3 + 32) >> 6;
    }
    wave_sync();
}

struct PicPtrs {
    uint8_t* y;
    uint8_t* u;
    uint8_t* v;
};

DEV PicPtrs out_planes(const h264r_batch& b, const Geom& g, int pic)
{
    PicPtrs p;
    p.y = b.out_y + (size_t)pic * g.ysz;
    p.u = b.out_u + (size_t)pic * g.csz;
    p.v = b.out_v + (size_t)pic * g.csz;
    return p;
}

// Plane of RefPicList[l][ri] (get_ref_pic dpb.cc:1046-1054); NULL for an index outside the
// list or an unloaded slot, so malformed input cannot fault the device.
DEV const uint8_t* ref_plane(const h264r_batch& b, const h264r_slice* sl, int l, int ri, int pl)
{
    if (ri >= H264R_MAX_REFS) return nullptr;
    int slot = sl->ref_slot[l][ri];
    if (slot < 0 || slot >= H264R_MAX_SLOTS) return nullptr;
    return b.ref_planes[slot * 3 + pl];
}

// I_PCM: mb_pred_ipcm decoder.cc:149-168.
DEV void pcm_mb(const h264r_mb& m, const int16_t* __restrict__ lv, const Geom& g, PicPtrs o, int mbx, int mby, int lane)
{
    const uint8_t* raw = reinterpret_cast<const uint8_t*>(lv);
    {
        int y = lane >> 2, x = (lane & 3) * 4;
        uint32_t v = *reinterpret_cast<const uint32_t*>(raw + y * 16 + x);
        *reinterpret_cast<uint32_t*>(o.y + (size_t)(mby * 16 + y) * g.W + mbx * 16 + x) = v;
    }
    {
        int pl = lane >> 5, y = (lane >> 2) & 7, x = (lane & 3) * 2;
        uint16_t v = *reinterpret_cast<const uint16_t*>(raw + 256 + pl * 64 + y * 8 + x);
        uint8_t* dst = pl ? o.v : o.u;
        *reinterpret_cast<uint16_t*>(dst + (size_t)(mby * 8 + y) * g.Wc + mbx * 8 + x) = v;
    }
}

// MB-level neighbour availability (get_neighbour + slice check + constrained intra,
// intra_prediction.cc:142-168 / 629-651 / 753-777).  Neighbours on earlier diagonals
// are always decoded.
DEV int nb_avail(const h264r_mb* mbs, const Geom& g, const h264r_mb& m, int cip, int nx, int ny)
{
    if (nx < 0 || ny < 0 || nx >= g.wmb || ny >= g.hmb) return 0;
    const h264r_mb* n = &mbs[ny * g.wmb + nx];
    if (n->slice != m.slice) return 0;
    if (cip && !(n->flags & H264R_MBF_INTRA)) return 0;
    return 1;
}

constexpr int TW = 28;   // LDS tile pitch: columns -1..23 (+pad), rows -1..15

struct IntraLds {
    ResLds R;
    uint8_t tile[17 * TW];           // luma: row -1 (cols -1..23), rows 0..15 (col -1 + MB)
    uint8_t ctile[2][9 * 12];        // chroma: row -1 (cols -1..7), rows 0..7 (col -1 + MB)
    int fs[2][33];                   // Intra8x8 filtered neighbours p(-1,-1), p(0..15,-1), p(-1,0..7)
};

DEV uint8_t& T(IntraLds& S, int x, int y) { return S.tile[(y + 1) * TW + (x + 1)]; }
DEV uint8_t& CT(IntraLds& S, int pl, int x, int y) { return S.ctile[pl][(y + 1) * 12 + (x + 1)]; }

// Intra4x4 / Intra8x8 sample prediction (intra_prediction.cc:189-346, 449-606) for one
// sample (x, y) of an NxN block; P(i, j) reads neighbour sample p(i, j).
template <int N, typename PF>
DEV int nxn_pred(int mode, int x, int y, int aA, int aB, PF P)
{
    constexpr int mHU = (N - 1) * 2 - 1;
    switch (mode) {
    case 0: return P(x, -1);
    case 1: return P(-1, y);
    case 2: {
        int sum = 0;
        if (aA || aB) {
            if (aA) for (int k = 0; k < N; ++k) sum += P(-1, k);
            if (aB) for (int k = 0; k < N; ++k) sum += P(k, -1);
            int sh = (N == 4 ? 1 : 2) + aA + aB;
            return (sum + (aA ? N / 2 : 0) + (aB ? N / 2 : 0)) >> sh;
        }
        return 128;
    }
    case 3:
        if (x == N - 1 && y == N - 1) return (P(x + y, -1) + 3 * P(x + y + 1, -1) + 2) >> 2;
        return (P(x + y, -1) + 2 * P(x + y + 1, -1) + P(x + y + 2, -1) + 2) >> 2;
    case 4:
        if (x > y) return (P(x - y - 2, -1) + 2 * P(x - y - 1, -1) + P(x - y, -1) + 2) >> 2;
        if (x < y) return (P(-1, y - x - 2) + 2 * P(-1, y - x - 1) + P(-1, y - x) + 2) >> 2;
        return (P(0, -1) + 2 * P(-1, -1) + P(-1, 0) + 2) >> 2;
    case 5: {
        int z = 2 * x - y;
        if (z >= 0 && (z & 1) == 0) return (P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 1) >> 1;
        if (z >= 0) return (P(x - (y >> 1) - 2, -1) + 2 * P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 2) >> 2;
        if (z == -1) return (P(-1, 0) + 2 * P(-1, -1) + P(0, -1) + 2) >> 2;
        return (P(-1, y - 2 * x - 1) + 2 * P(-1, y - 2 * x - 2) + P(-1, y - 2 * x - 3) + 2) >> 2;
    }
    case 6: {
        int z = 2 * y - x;
        if (z >= 0 && (z & 1) == 0) return (P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 1) >> 1;
        if (z >= 0) return (P(-1, y - (x >> 1) - 2) + 2 * P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 2) >> 2;
        if (z == -1) return (P(-1, 0) + 2 * P(-1, -1) + P(0, -1) + 2) >> 2;
        return (P(x - 2 * y - 1, -1) + 2 * P(x - 2 * y - 2, -1) + P(x - 2 * y - 3, -1) + 2) >> 2;
    }
    case 7:
        if ((y & 1) == 0) return (P(x + (y >> 1), -1) + P(x + (y >> 1) + 1, -1) + 1) >> 1;
        return (P(x + (y >> 1), -1) + 2 * P(x + (y >> 1) + 1, -1) + P(x + (y >> 1) + 2, -1) + 2) >> 2;
    default: {
        int z = x + 2 * y;
        if (z < mHU && (z & 1) == 0) return (P(-1, y + (x >> 1)) + P(-1, y + (x >> 1) + 1) + 1) >> 1;
        if (z < mHU) return (P(-1, y + (x >> 1)) + 2 * P(-1, y + (x >> 1) + 1) + P(-1, y + (x >> 1) + 2) + 2) >> 2;
        if (z == mHU) return (P(-1, N - 2) + 3 * P(-1, N - 1) + 2) >> 2;
        return P(-1, N - 1);
    }
    }
}

// Intra MB (mbx, mby) of picture `pic` (no-op for inter / I_PCM MBs); one wave.
DEV void intra_mb(const h264r_batch& b, const Geom& g, int pic, int mbx, int mby, int lane, IntraLds& S)
{
    const int a = mby * g.wmb + mbx;
    const h264r_mb* mbs = b.mbs + (size_t)pic * g.nmb;
    const h264r_mb m = load_mb(&mbs[a]);
    if (!mb_is_intra(m) || m.mb_type == H264R_I_PCM) return;

    const int cip = b.pics[pic].constrained_intra_pred;
    const PicPtrs o = out_planes(b, g, pic);
    const int16_t* lv = b.levels + m.coef_off;
    const int avA = nb_avail(mbs, g, m, cip, mbx - 1, mby), avB = nb_avail(mbs, g, m, cip, mbx, mby - 1);
    const int avC = nb_avail(mbs, g, m, cip, mbx + 1, mby - 1), avD = nb_avail(mbs, g, m, cip, mbx - 1, mby - 1);

    // ---- neighbour samples into the LDS tiles (only what is available is read)
    {
        const int X = mbx * 16, Y = mby * 16;
        for (int k = lane; k < 25; k += 64) {            // row -1, cols -1..23
            int x = k - 1;
            int ok = x < 0 ? avD : (x < 16 ? avB : avC);
            T(S, x, -1) = ok ? o.y[(size_t)(Y - 1) * g.W + X + x] : 0;
        }
        if (lane < 16) T(S, -1, lane) = avA ? o.y[(size_t)(Y + lane) * g.W + X - 1] : 0;
        if (lane >= 32 && lane < 50) {                   // chroma: 9 top + 8 left per plane
            int k = lane - 32, pl = k / 9, i = k % 9;
            const uint8_t* cp = pl ? o.v : o.u;
            const int Xc = mbx * 8, Yc = mby * 8;
            int x = i - 1;
            CT(S, pl, x, -1) = (x < 0 ? avD : avB) ? cp[(size_t)(Yc - 1) * g.Wc + Xc + x] : 0;
            if (i < 8) CT(S, pl, -1, i) = avA ? cp[(size_t)(Yc + i) * g.Wc + Xc - 1] : 0;
        }
    }
    residual_mb(m, lv, &b.quant[pic], S.R, lane);     // includes wave_sync

    const int cbpl = m.cbp & 15;
    if (m.mb_type == H264R_I_16x16) {
        // Intra16x16 (intra_prediction.cc:668-735) + construction_16x16 (transform.cc:940-959)
        const int mode = m.i16_mode;
        int dc = 128, pb = 0, pc = 0, pa = 0;
        if (mode == 2 && (avA || avB)) {
            int sum = 0;
            if (avA) for (int k = 0; k < 16; ++k) sum += T(S, -1, k);
            if (avB) for (int k = 0; k < 16; ++k) sum += T(S, k, -1);
            dc = (sum + (avA ? 8 : 0) + (avB ? 8 : 0)) >> (3 + avA + avB);
        }
        if (mode == 3) {
            int Hs = 0, Vs = 0;
            for (int x = 0; x < 8; ++x) Hs += (x + 1) * (T(S, 8 + x, -1) - T(S, 6 - x, -1));
            for (int y = 0; y < 8; ++y) Vs += (y + 1) * (T(S, -1, 8 + y) - T(S, -1, 6 - y));
            pa = 16 * (T(S, -1, 15) + T(S, 15, -1));
            pb = (5 * Hs + 32) >> 6; pc = (5 * Vs + 32) >> 6;
        }
        int y = lane >> 2, x0 = (lane & 3) * 4;
        uint32_t w = 0;
        for (int c = 0; c < 4; ++c) {
            int x = x0 + c, p;
            if (mode == 0) p = T(S, x, -1);
            else if (mode == 1) p = T(S, -1, y);
            else if (mode == 2) p = dc;
            else p = clip255((pa + pb * (x - 7) + pc * (y - 7) + 16) >> 5);
            w |= (uint32_t)clip255(p + S.R.lum[y][x]) << (8 * c);
        }
        *reinterpret_cast<uint32_t*>(o.y + (size_t)(mby * 16 + y) * g.W + mbx * 16 + x0) = w;
    } else if (m.mb_type == H264R_I_8x8) {
        for (int blk = 0; blk < 4; ++blk) {
            const int xO = (blk & 1) * 8, yO = (blk >> 1) * 8;
            const int aA = xO > 0 ? 1 : avA, aB = yO > 0 ? 1 : avB;
            const int aD = (xO > 0 && yO > 0) ? 1 : (xO == 0 && yO == 0) ? avD : (xO == 0 ? avA : avB);
            int aC = yO > 0 ? (xO == 0) : (xO == 0 ? avB : avC);   // :370-376
            const int mode = (m.ipred[blk >> 1] >> ((blk & 1) * 4)) & 15;
            // Intra8x8::filtering (intra_prediction.cc:413-447) -> fs
            int* fs = S.fs[blk & 1];
            auto po = [&](int x, int y) -> int {
                if (y < 0 && x >= 8 && !aC) x = 7;        // p(x,-1) substitution :404-407
                return T(S, xO + x, yO + y);
            };
            if (lane < 33) {
                int v = 0;
                if (lane == 0) {                            // p(-1,-1)
                    if (aD) {
                        if (aA && aB) v = (po(0, -1) + 2 * po(-1, -1) + po(-1, 0) + 2) >> 2;
                        else if (aB) v = (3 * po(-1, -1) + po(0, -1) + 2) >> 2;
                        else if (aA) v = (3 * po(-1, -1) + po(-1, 0) + 2) >> 2;
                        else v = po(-1, -1);
                    }
                } else if (lane <= 16) {                    // p(x,-1), x = lane-1
                    int x = lane - 1;
                    if (aB) {
                        if (x == 0) v = aD ? (po(-1, -1) + 2 * po(0, -1) + po(1, -1) + 2) >> 2 : (3 * po(0, -1) + po(1, -1) + 2) >> 2;
                        else if (x < 15) v = (po(x - 1, -1) + 2 * po(x, -1) + po(x + 1, -1) + 2) >> 2;
                        else v = (po(14, -1) + 3 * po(15, -1) + 2) >> 2;
                    }
                } else if (lane <= 24) {                    // p(-1,y), y = lane-17
                    int y = lane - 17;
                    if (aA) {
                        if (y == 0) v = aD ? (po(-1, -1) + 2 * po(-1, 0) + po(-1, 1) + 2) >> 2 : (3 * po(-1, 0) + po(-1, 1) + 2) >> 2;
                        else if (y < 7) v = (po(-1, y - 1) + 2 * po(-1, y) + po(-1, y + 1) + 2) >> 2;
                        else v = (po(-1, 6) + 3 * po(-1, 7) + 2) >> 2;
                    }
                }
                fs[lane] = v;
            }
            wave_sync();
            auto P = [&](int x, int y) -> int { return y < 0 ? (x < 0 ? fs[0] : fs[1 + x]) : fs[17 + y]; };
            {
                int x = lane & 7, y = lane >> 3;
                int p = nxn_pred<8>(mode, x, y, aA, aB, P);
                int v = (cbpl >> blk) & 1 ? clip255(p + S.R.lum[yO + y][xO + x]) : p;
                T(S, xO + x, yO + y) = (uint8_t)v;
            }
            wave_sync();
        }
    } else {   // I_4x4
        for (int bk = 0; bk < 16; ++bk) {
            const int xO = ((bk / 4) % 2) * 8 + ((bk % 4) % 2) * 4;
            const int yO = ((bk / 4) / 2) * 8 + ((bk % 4) / 2) * 4;
            const int aA = xO > 0 ? 1 : avA, aB = yO > 0 ? 1 : avB;
            int aC;
            if (yO == 0) aC = xO + 4 < 16 ? avB : avC;
            else aC = (xO + 4 < 16) && !(xO == 4 && (yO == 4 || yO == 12));   // :154
            const int mode = (m.ipred[bk >> 1] >> ((bk & 1) * 4)) & 15;
            if (lane < 16) {
                int x = lane & 3, y = lane >> 2;
                auto P = [&](int i, int j) -> int {
                    if (j < 0 && i >= 4 && !aC) i = 3;       // :183-185
                    return T(S, xO + i, yO + j);
                };
                int p = nxn_pred<4>(mode, x, y, aA, aB, P);
                int v = (cbpl >> ((yO / 8) * 2 + xO / 8)) & 1 ? clip255(p + S.R.lum[yO + y][xO + x]) : p;
                T(S, xO + x, yO + y) = (uint8_t)v;
            }
            wave_sync();
        }
    }
    if (m.mb_type != H264R_I_16x16) {
        int y = lane >> 2, x0 = (lane & 3) * 4;
        uint32_t w = 0;
        for (int c = 0; c < 4; ++c) w |= (uint32_t)T(S, x0 + c, y) << (8 * c);
        *reinterpret_cast<uint32_t*>(o.y + (size_t)(mby * 16 + y) * g.W + mbx * 16 + x0) = w;
    }

    // ---- chroma: IntraPrediction::Chroma (intra_prediction.cc:748-894) + construction_chroma
    {
        const int pl = lane >> 5, y = (lane >> 2) & 7, x0 = (lane & 3) * 2;
        const int mode = m.chroma_mode;
        uint32_t w = 0;
        for (int c = 0; c < 2; ++c) {
            int x = x0 + c, p;
            if (mode == 0) {
                int xO = x & 4, yO = y & 4, aA, aB;
                if ((xO == 0 && yO == 0) || (xO > 0 && yO > 0)) { aA = avA; aB = avB; }
                else if (xO > 0) { aA = avB ? 0 : avA; aB = avB; }
                else { aA = avA; aB = avA ? 0 : avB; }
                int sum = 0;
                if (aA || aB) {
                    if (aA) for (int k = 0; k < 4; ++k) sum += CT(S, pl, -1, yO + k);
                    if (aB) for (int k = 0; k < 4; ++k) sum += CT(S, pl, xO + k, -1);
                    p = (sum + (aA ? 2 : 0) + (aB ? 2 : 0)) >> (1 + aA + aB);
                } else p = 128;
            } else if (mode == 1) p = CT(S, pl, -1, y);
            else if (mode == 2) p = CT(S, pl, x, -1);
            else {
                int Hs = 0, Vs = 0;
                for (int k = 0; k < 4; ++k) Hs += (k + 1) * (CT(S, pl, 4 + k, -1) - CT(S, pl, 2 - k, -1));
                for (int k = 0; k < 4; ++k) Vs += (k + 1) * (CT(S, pl, -1, 4 + k) - CT(S, pl, -1, 2 - k));
                int pa = 16 * (CT(S, pl, -1, 7) + CT(S, pl, 7, -1));
                int pb = (34 * Hs + 32) >> 6, pc = (34 * Vs + 32) >> 6;
                p = clip255((pa + pb * (x - 3) + pc * (y - 3) + 16) >> 5);
            }
            w |= (uint32_t)clip255(p + S.R.chr[pl][y][x]) << (8 * c);
        }
        uint8_t* dst = pl ? o.v : o.u;
        *reinterpret_cast<uint16_t*>(dst + (size_t)(mby * 8 + y) * g.Wc + mbx * 8 + x0) = (uint16_t)w;
    }
}

}  // namespace h264r
