// device_common.h -- shared device helpers of the gfx950 reconstruction kernels.
//
// Canonical formats are those of include/h264r.h.  Every helper cites the
// reference lines whose arithmetic it reproduces (H/ = R/src/codec/h264/).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "h264r.h"

#define DEV __device__ __forceinline__

namespace h264r {

// --------------------------------------------------------------------- geometry
struct Geom {
    int wmb, hmb;          // picture size in MBs
    int W, H, Wc, Hc;      // plane sizes in samples
    int W4, H4;            // 4x4-block grid
    int nmb;               // W*H MBs
    size_t ysz, csz;       // plane sizes in bytes
    int motion_plane;      // 4x4 entries per list
};

DEV Geom make_geom(int wmb, int hmb)
{
    Geom g;
    g.wmb = wmb; g.hmb = hmb;
    g.W = wmb * 16; g.H = hmb * 16; g.Wc = wmb * 8; g.Hc = hmb * 8;
    g.W4 = wmb * 4; g.H4 = hmb * 4;
    g.nmb = wmb * hmb;
    g.ysz = (size_t)g.W * g.H; g.csz = (size_t)g.Wc * g.Hc;
    g.motion_plane = g.W4 * g.H4;
    return g;
}

DEV int clip3(int lo, int hi, int x) { return x < lo ? lo : (x > hi ? hi : x); }   // defines.h:48-52
DEV int clip255(int x) { return clip3(0, 255, x); }                                 // clip1, defines.h:54-58
DEV int iabs(int x) { return x < 0 ? -x : x; }

// Load the 32-byte MB record into SGPR-friendly registers (wave-uniform address).
DEV h264r_mb load_mb(const h264r_mb* p)
{
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4 a = q[0], b = q[1];
    h264r_mb m;
    uint32_t* w = reinterpret_cast<uint32_t*>(&m);
    w[0] = __builtin_amdgcn_readfirstlane(a.x); w[1] = __builtin_amdgcn_readfirstlane(a.y);
    w[2] = __builtin_amdgcn_readfirstlane(a.z); w[3] = __builtin_amdgcn_readfirstlane(a.w);
    w[4] = __builtin_amdgcn_readfirstlane(b.x); w[5] = __builtin_amdgcn_readfirstlane(b.y);
    w[6] = __builtin_amdgcn_readfirstlane(b.z); w[7] = __builtin_amdgcn_readfirstlane(b.w);
    return m;
}

// Scalar (constant address space) load of data that no kernel of the batch writes
// (MB records, slice headers): a wave-uniform address becomes an s_load, issued back
// to back with the others and waited on lgkmcnt, not interleaved with vmcnt waits.
DEV uint32_t ld_const(const void* p) { return *(const __attribute__((address_space(4))) uint32_t*)p; }
DEV h264r_mb load_mb_const(const h264r_mb* p)
{
    h264r_mb m;
    uint32_t* w = reinterpret_cast<uint32_t*>(&m);
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = ld_const(reinterpret_cast<const uint32_t*>(p) + i);
    return m;
}

// Wave-level barrier for LDS scratch owned by one wave: orders this wave's LDS
// accesses across lanes without a workgroup barrier (other waves of the
// workgroup run independent work).  H264R_SYNC_NODRAIN drops the lgkmcnt(0)
// drain: a wave's LDS instructions execute in issue order, so only the compiler
// has to be kept from moving accesses across the barrier (measurement variant).
DEV void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#ifndef H264R_SYNC_NODRAIN
    __builtin_amdgcn_s_waitcnt(0xc07f);          // lgkmcnt(0): LDS ops of this wave done
#endif
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

DEV int mb_is_intra(const h264r_mb& m) { return (m.flags & H264R_MBF_INTRA) != 0; }

// ----------------------------------------------------------- level block layout
// Section offsets of the compacted level block (include/h264r.h), int16 units.
struct LevelOffs {
    int b8[4];      // -1 if not coded
    int cac, ldc, cdc;
};

// Offset of coded 8x8 luma block k inside the level block, or -1 (register-only form
// of LevelOffs::b8 for a per-lane k).
DEV int b8_offset(int cbp, int k)
{
    const int cbpl = cbp & 15;
    return (cbpl >> k) & 1 ? 64 * __builtin_popcount(cbpl & ((1 << k) - 1)) : -1;
}

DEV LevelOffs level_offsets(const h264r_mb& m)
{
    LevelOffs o;
    int p = 0, cbpl = m.cbp & 15, cbpc = m.cbp >> 4;
    for (int k = 0; k < 4; ++k) { o.b8[k] = (cbpl >> k) & 1 ? p : -1; p += ((cbpl >> k) & 1) * 64; }
    o.cac = cbpc == 2 ? p : -1; p += cbpc == 2 ? 128 : 0;
    o.ldc = m.mb_type == H264R_I_16x16 ? p : -1; p += m.mb_type == H264R_I_16x16 ? 16 : 0;
    o.cdc = cbpc ? p : -1;
    return o;
}

// ----------------------------------------------------------- residual (transform.cc)
// Dequantise one 4x4 AC/luma level, inverse_quantize transform.cc:394-413.
DEV int dq4(int lev, int scale, int per) { return ((lev * scale) * (1 << per) + 8) >> 4; }
// 8x8: transform.cc:414-419.
DEV int dq8(int lev, int scale, int per) { return ((lev * scale) * (1 << per) + 32) >> 6; }

// 1-D 4-point inverse core transform, rows of inverse_4x4 (transform.cc:602-617).
DEV void idct4(int d0, int d1, int d2, int d3, int& o0, int& o1, int& o2, int& o3)
{
    int e0 = d0 + d2, e1 = d0 - d2, e2 = (d1 >> 1) - d3, e3 = d1 + (d3 >> 1);
    o0 = e0 + e3; o1 = e1 + e2; o2 = e1 - e2; o3 = e0 - e3;
}

// 1-D 8-point inverse transform (transform.cc:658-683).
DEV void idct8(const int* in, int* out)
{
    int e0 = in[0] + in[4];
    int e1 = -in[3] + in[5] - in[7] - (in[7] >> 1);
    int e2 = in[0] - in[4];
    int e3 = in[1] + in[7] - in[3] - (in[3] >> 1);
    int e4 = (in[2] >> 1) - in[6];
    int e5 = -in[1] + in[7] + in[5] + (in[5] >> 1);
    int e6 = in[2] + (in[6] >> 1);
    int e7 = in[3] + in[5] + in[1] + (in[1] >> 1);
    int f0 = e0 + e6, f1 = e1 + (e7 >> 2), f2 = e2 + e4, f3 = e3 + (e5 >> 2);
    int f4 = e2 - e4, f5 = (e3 >> 2) - e5, f6 = e0 - e6, f7 = e7 - (e1 >> 2);
    out[0] = f0 + f7; out[1] = f2 + f5; out[2] = f4 + f3; out[3] = f6 + f1;
    out[4] = f6 - f1; out[5] = f4 - f3; out[6] = f2 - f5; out[7] = f0 - f7;
}

// ---------------------------------------------------------------- motion comp.
// Clamped sample fetch (equivalent to the reference's padded planes, picture.cc:182-205).
DEV int pxl(const uint8_t* __restrict__ img, int W, int H, int x, int y)
{
    return img[clip3(0, H - 1, y) * W + clip3(0, W - 1, x)];
}
DEV int tap6(int a, int b, int c, int d, int e, int f) { return a - 5 * b + 20 * c + 20 * d - 5 * e + f; }

// ------------------------------------------------------------ row-window MC
// The per-sample forms above fetch one byte per tap.  The MC path proper loads
// each reference row as three aligned dwords and extracts the samples it needs;
// clamping (the padded-plane equivalence of inter_prediction.cc:185-186) is
// applied to the row index always and to the column only for windows that
// cross the picture edge.  Reads may run up to 11 bytes past the last sample
// of a row: reference planes carry H264R_PLANE_SLACK bytes of slack.

// Samples ref(x-2+k, y), k = 0..8, of the row whose dwords w0..w2 start at
// a = clip(x-2) & ~3.
DEV void row9(uint32_t w0, uint32_t w1, uint32_t w2, int x, int W, int (&p)[9])
{
    if (x - 2 >= 0 && x + 6 < W) {
        const int s = (x - 2) & 3;
        const uint32_t r0 = __builtin_amdgcn_alignbyte(w1, w0, s);
        const uint32_t r1 = __builtin_amdgcn_alignbyte(w2, w1, s);
#pragma unroll
        for (int k = 0; k < 4; ++k) { p[k] = (r0 >> (8 * k)) & 255; p[4 + k] = (r1 >> (8 * k)) & 255; }
        p[8] = (w2 >> (8 * s)) & 255;
    } else {
        const int a = clip3(0, W - 1, x - 2) & ~3;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int idx = clip3(0, W - 1, x - 2 + k) - a;
            const uint32_t d = idx < 4 ? w0 : (idx < 8 ? w1 : w2);
            p[k] = (d >> (8 * (idx & 3))) & 255;
        }
    }
}

// Global-address-space view of a pointer whose address space the compiler cannot
// infer (a plane pointer read from LDS or picked per lane): loads through it are
// `global_load`, not `flat_load`.  A flat load counts on lgkmcnt as well as vmcnt and
// may return out of order, so every later LDS wait -- and every use of any load --
// would also wait for it (a prefetch would stop overlapping anything).
typedef const uint32_t __attribute__((address_space(1))) gdword;
DEV const gdword* as_global(const void* p) { return (const gdword*)p; }
template <typename T>
DEV T load_global(const void* p) { return *(const __attribute__((address_space(1))) T*)p; }

DEV const gdword* row_dwords(const uint8_t* __restrict__ img, int W, int H, int x, int y)
{
    const int a = clip3(0, W - 1, x - 2) & ~3;
    return as_global(img + (size_t)clip3(0, H - 1, y) * W + a);
}

// Four luma prediction samples (x..x+3, y) at quarter-sample phase (xf, yf),
// get_block_luma (inter_prediction.cc:158-340) in spec form (8.4.2.2.1): the
// half-sample values b (horizontal), h (vertical), j (centre) and their
// averages.  The 6 rows y-2..y+3 are streamed; each tap row is loaded once.
// XF/YF >= 0 fix the phase at compile time (wave-uniform MV phase: only that
// case's arithmetic is emitted); -1 takes it from xf_rt/yf_rt per lane.
template <int XF = -1, int YF = -1>
DEV void luma_pred4(const uint8_t* __restrict__ img, int W, int H, int x, int y, int xf_rt, int yf_rt, int (&out)[4])
{
    constexpr int C6[6] = {1, -5, 20, 20, -5, 1};
    const int xf = XF >= 0 ? XF : xf_rt, yf = YF >= 0 ? YF : yf_rt;
    if (yf == 0) {                                    // G, a, b, c: one row
        const gdword* q = row_dwords(img, W, H, x, y);
        int p[9];
        row9(q[0], q[1], q[2], x, W, p);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (xf == 0) { out[c] = p[2 + c]; continue; }
            const int b = clip255((tap6(p[c], p[c + 1], p[c + 2], p[c + 3], p[c + 4], p[c + 5]) + 16) >> 5);
            out[c] = xf == 2 ? b : (b + (xf == 3 ? p[3 + c] : p[2 + c]) + 1) >> 1;
        }
        return;
    }
    uint32_t w[6][3];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const gdword* q = row_dwords(img, W, H, x, y - 2 + k);
        w[k][0] = q[0]; w[k][1] = q[1]; w[k][2] = q[2];
    }
    const bool jfam = xf == 2 || (yf == 2 && xf != 0);   // needs the centre sample j
    const int hs = xf == 3 ? 1 : 0;                        // column of h / G for odd phases
    const int brow = yf == 3 ? 3 : 2;                      // row of b / G (y or y+1)
    int hacc[4] = {0, 0, 0, 0}, jacc[4] = {0, 0, 0, 0}, bsv[4] = {0, 0, 0, 0}, gsv[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        int p[9];
        row9(w[k][0], w[k][1], w[k][2], x, W, p);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            hacc[c] += C6[k] * (hs ? p[3 + c] : p[2 + c]);
            if (k == brow) gsv[c] = p[2 + c];
            if (jfam || ((xf & 1) && k == brow)) {
                const int b1 = tap6(p[c], p[c + 1], p[c + 2], p[c + 3], p[c + 4], p[c + 5]);
                jacc[c] += C6[k] * b1;
                if (k == brow) bsv[c] = b1;
            }
        }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int h = clip255((hacc[c] + 16) >> 5);
        const int b = clip255((bsv[c] + 16) >> 5);
        int v;
        if (xf == 0) v = yf == 2 ? h : (h + gsv[c] + 1) >> 1;                 // d, h, n
        else if (!jfam) v = (b + h + 1) >> 1;                                 // e, g, p, r
        else {
            const int j = clip255((jacc[c] + 512) >> 10);
            if (xf == 2 && yf == 2) v = j;                                    // j
            else if (xf == 2) v = (j + b + 1) >> 1;                           // f, q
            else v = (j + h + 1) >> 1;                                        // i, k
        }
        out[c] = v;
    }
}

// Two chroma prediction samples (xi, xi+1; yi) at eighth-sample phase (xf, yf),
// get_block_chroma (inter_prediction.cc:380-404).
DEV void chroma_pred2(const uint8_t* __restrict__ img, int W, int H, int xi, int yi, int xf, int yf, int (&out)[2])
{
    const int a = clip3(0, W - 1, xi) & ~3;
    int p[2][3];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const gdword* q = as_global(img + (size_t)clip3(0, H - 1, yi + k) * W + a);
        const uint32_t w0 = q[0], w1 = q[1];
        if (xi >= 0 && xi + 2 < W) {
            const uint32_t r = __builtin_amdgcn_alignbyte(w1, w0, xi & 3);
            p[k][0] = r & 255; p[k][1] = (r >> 8) & 255; p[k][2] = (r >> 16) & 255;
        } else {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int idx = clip3(0, W - 1, xi + c) - a;
                p[k][c] = ((idx < 4 ? w0 : w1) >> (8 * (idx & 3))) & 255;
            }
        }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
        out[c] = ((8 - xf) * (8 - yf) * p[0][c] + xf * (8 - yf) * p[0][c + 1] + (8 - xf) * yf * p[1][c] +
                  xf * yf * p[1][c + 1] + 32) >> 6;
}

DEV int rshift_rnd(int x, int a) { return a > 0 ? (x + (1 << (a - 1))) >> a : x; }  // inter_prediction.cc:35-38

// mc_prediction / bi_prediction combine (inter_prediction.cc:53-156) for one sample.
DEV int wp_combine(const h264r_slice* __restrict__ sl, int dir, int r0, int r1, int v0, int v1, int pl)
{
    int mode = sl->wp_mode;
    if (dir != 2) {
        if (mode != 1) return dir == 0 ? v0 : v1;
        int r = dir == 0 ? r0 : r1, v = dir == 0 ? v0 : v1;
        int w = sl->wp_weight[dir][r][pl], o = sl->wp_offset[dir][r][pl];
        int d = pl ? sl->chroma_log2_wd : sl->luma_log2_wd;
        return clip255(rshift_rnd(w * v, d) + o);
    }
    if (mode == 0) return (v0 + v1 + 1) >> 1;
    int w0, w1, o0, o1;
    if (mode == 1) {
        w0 = sl->wp_weight[0][r0][pl]; w1 = sl->wp_weight[1][r1][pl];
        o0 = sl->wp_offset[0][r0][pl]; o1 = sl->wp_offset[1][r1][pl];
    } else {
        w1 = sl->implicit_w1[r0][r1]; w0 = 64 - w1; o0 = o1 = 0;
    }
    int d = (pl ? sl->chroma_log2_wd : sl->luma_log2_wd) + 1;
    return clip255(rshift_rnd(w0 * v0 + w1 * v1, d) + ((o0 + o1 + 1) >> 1));
}

// ---------------------------------------------------------------- deblocking
// Tables 8-16 / 8-17 (deblock.cc:294-324), packed alpha | beta<<8 | tc0[3]<<16.. in one word.
__device__ static const uint32_t DB_AB[52] = {
#define AB(a, b) ((uint32_t)(a) | ((uint32_t)(b) << 8))
    AB(0, 0), AB(0, 0), AB(0, 0), AB(0, 0), AB(0, 0), AB(0, 0), AB(0, 0), AB(0, 0), AB(0, 0), AB(0, 0),
    AB(0, 0), AB(0, 0), AB(0, 0), AB(0, 0), AB(0, 0), AB(0, 0), AB(4, 2), AB(4, 2), AB(5, 2), AB(6, 3),
    AB(7, 3), AB(8, 3), AB(9, 3), AB(10, 4), AB(12, 4), AB(13, 4), AB(15, 6), AB(17, 6), AB(20, 7), AB(22, 7),
    AB(25, 8), AB(28, 8), AB(32, 9), AB(36, 9), AB(40, 10), AB(45, 10), AB(50, 11), AB(56, 11), AB(63, 12), AB(71, 12),
    AB(80, 13), AB(90, 13), AB(101, 14), AB(113, 14), AB(127, 15), AB(144, 15), AB(162, 16), AB(182, 16), AB(203, 17), AB(226, 17),
    AB(255, 18), AB(255, 18)
#undef AB
};
__device__ static const uint32_t DB_TC0[52] = {
#define T(a, b, c) ((uint32_t)(a) | ((uint32_t)(b) << 8) | ((uint32_t)(c) << 16))
    T(0, 0, 0), T(0, 0, 0), T(0, 0, 0), T(0, 0, 0), T(0, 0, 0), T(0, 0, 0), T(0, 0, 0), T(0, 0, 0),
    T(0, 0, 0), T(0, 0, 0), T(0, 0, 0), T(0, 0, 0), T(0, 0, 0), T(0, 0, 0), T(0, 0, 0), T(0, 0, 0),
    T(0, 0, 0), T(0, 0, 1), T(0, 0, 1), T(0, 0, 1), T(0, 0, 1), T(0, 1, 1), T(0, 1, 1), T(1, 1, 1),
    T(1, 1, 1), T(1, 1, 1), T(1, 1, 1), T(1, 1, 2), T(1, 1, 2), T(1, 1, 2), T(1, 1, 2), T(1, 2, 3),
    T(1, 2, 3), T(2, 2, 3), T(2, 2, 4), T(2, 3, 4), T(2, 3, 4), T(3, 3, 5), T(3, 4, 6), T(3, 4, 6),
    T(4, 5, 7), T(4, 5, 8), T(4, 6, 9), T(5, 7, 10), T(6, 8, 11), T(6, 8, 13), T(7, 10, 14), T(8, 11, 16),
    T(9, 12, 18), T(10, 13, 20), T(11, 15, 23), T(13, 17, 25)
#undef T
};

// filter_strong / filter_normal (deblock.cc:327-415) on 8 samples p3..p0 q0..q3 held in
// registers; returns the updated samples in place.
DEV void filter_samples(int& p3, int& p2, int& p1, int& p0, int& q0, int& q1, int& q2, int& q3,
                        int alpha, int beta, int bS, int chroma, int tc0)
{
    if (!(iabs(p0 - q0) < alpha && iabs(p1 - p0) < beta && iabs(q1 - q0) < beta)) return;
    int ap = iabs(p2 - p0), aq = iabs(q2 - q0);
    if (bS == 4) {
        int np0, np1, np2, nq0, nq1, nq2;
        int strong = iabs(p0 - q0) < (alpha >> 2) + 2;
        if (!chroma && ap < beta && strong) {
            np0 = (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3;
            np1 = (p2 + p1 + p0 + q0 + 2) >> 2;
            np2 = (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3;
        } else { np0 = (2 * p1 + p0 + q1 + 2) >> 2; np1 = p1; np2 = p2; }
        if (!chroma && aq < beta && strong) {
            nq0 = (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3;
            nq1 = (p0 + q0 + q1 + q2 + 2) >> 2;
            nq2 = (2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3;
        } else { nq0 = (2 * q1 + q0 + p1 + 2) >> 2; nq1 = q1; nq2 = q2; }
        p0 = np0; p1 = np1; p2 = np2; q0 = nq0; q1 = nq1; q2 = nq2;
    } else {
        int tc = chroma ? tc0 + 1 : tc0 + (ap < beta) + (aq < beta);
        int delta = clip3(-tc, tc, (((q0 - p0) * 4) + (p1 - q1) + 4) >> 3);
        int np1 = p1, nq1 = q1;
        if (!chroma && ap < beta) np1 = p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 * 2)) >> 1);
        if (!chroma && aq < beta) nq1 = q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 * 2)) >> 1);
        p0 = clip255(p0 + delta); q0 = clip255(q0 - delta);
        p1 = np1; q1 = nq1;
    }
}

}  // namespace h264r
