// mb_inter4.h -- inter (and I_PCM) macroblocks, FOUR per 64-lane wave, one lane per
// 4x4 luma block (+ its 2x2 chroma sub-blocks in both planes), and the deblocking
// record of every MB.
//
//   Decoder::mb_pred_inter decoder.cc:212-262 (partition walk = per-4x4 motion),
//   InterPrediction::get_block_luma inter_prediction.cc:158-340 (6-tap qpel),
//   get_block_chroma :342-406 (bilinear), mc_prediction :53-86 and bi_prediction
//   :88-156 (weighted prediction), Transform::inverse_transform_inter
//   transform.cc:1051-1095 (inverse_4x4 :597-641, inverse_8x8 :643-733, chroma DC
//   :875-889, construction :913-984), mb_pred_ipcm decoder.cc:149-168,
//   Deblock::strength deblock.cc:78-289 (boundary strengths, DbInfo).
//
// Why this shape: a wave per MB with a lane per sample row keeps one MB in flight
// per wave, recomputes the 6-tap intermediates of every row in every lane, and
// leaves the kernel latency-bound (a handful of dependent global round trips per MB,
// at 5 waves per SIMD).  With a lane per 4x4 block a wave carries four MBs, each
// lane filters its 9x9 reference window once (the horizontal intermediates of a row
// feed both the half-sample b and the centre j of all four output rows), the 4x4
// inverse transform runs entirely in-lane, and a 4x4 block's motion is exactly what
// the boundary strengths of its left and top edges need.
//
// Lane roles: g = lane >> 4 picks the MB (a0 + g), blk = lane & 15 the 4x4 block in
// raster order (bx = blk & 3, by = blk >> 2).  Chroma: the lane owns the 2x2 chroma
// samples (2bx.., 2by..) of each plane (4:2:0: the chroma of a luma 4x4 block, with
// the same motion vector).  A chroma 4x4 transform block is spread over the lanes
// {blk, blk^1, blk^4, blk^5}; an 8x8 luma transform block likewise.
#pragma once
#include "mb_deblock.h"

// H264R_INTER_DIAG: diagnostic builds only (wrong output; make EXTRA=-DH264R_INTER_DIAG=<bits>) that
// take one part of k_inter4r away to time the rest: 1 one 16-byte store per lane, 2 no luma
// filter (window loads kept), 4 neither, 8 no chroma MC, 16 no residual (nor its loads), 32 no
// deblocking records, 64 no luma residual transform (its loads kept), 128 the same for chroma
#ifndef H264R_INTER_DIAG
#define H264R_INTER_DIAG 0
#endif

namespace h264r {

constexpr int INTER4_MBS = 16;   // MBs per 256-thread workgroup (4 waves x 4)
constexpr int INTER4_LDS_SLICES = 64;   // slices whose ref tables the workgroup keeps in LDS

struct Inter4Lds {
    const uint8_t* planes[3 * H264R_MAX_SLOTS];
    uint2 hdr[INTER4_LDS_SLICES];                            // dwords 0..1 of the picture's slices (type, idc, offsets, wp)
    int8_t ref_slot[INTER4_LDS_SLICES][2][H264R_MAX_REFS];   // h264r_slice::ref_slot of the picture's slices
    uint8_t slice_type[INTER4_LDS_SLICES];                   // h264r_slice::slice_type of the same slices
};

// Byte `off` of slice `slice`'s h264r_slice, for the slices past the LDS copy: a buffer
// load (a select between an LDS and a global byte became one flat load, whose wait covers
// every outstanding load of both kinds).
DEV int slice_byte(const h264r_slice* slices, int slice, int off)
{
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<h264r_slice*>(slices + slice), 0,
                                                                        (int)sizeof(h264r_slice), 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b8(rs, off, 0, 0);
}
// slice_type of a slice: the LDS copy, else the slice table
DEV int slice_type_of(const h264r_slice* slices, const Inter4Lds& S, int slice)
{
    int t = S.slice_type[min(slice, INTER4_LDS_SLICES - 1)];
    if (slice >= INTER4_LDS_SLICES) t = slice_byte(slices, slice, (int)offsetof(h264r_slice, slice_type));
    return t;
}

// Dwords 0..1 of slice `slice` (type, idc, filter offsets, wp mode, log2 wd): the LDS copy,
// else the slice table
DEV uint2 slice_hdr(const h264r_slice* slices, const Inter4Lds& S, int slice)
{
    if (slice < INTER4_LDS_SLICES) return S.hdr[slice];
    return *reinterpret_cast<const uint2*>(&slices[slice]);
}

// Motion of one 4x4 block as {mv, ref_idx | slot << 8} per list: RefPicList[l][ref_idx]
// of the block's slice resolved to its DPB slot (get_ref_pic dpb.cc:1046-1054;
// pic_motion_params::ref_pic interpret_mb.cc:611-623), slot -1 when the list is unused.
DEV uint2 motion_word(uint32_t mv, int ri, const h264r_slice* slices, const Inter4Lds& S, int slice, int l)
{
    // the table read at a clamped index and the "no list" case selected afterwards: an LDS
    // read under the lane's `has` compiled to a lane-divergent branch
    const bool has = ri >= 0 && ri < H264R_MAX_REFS;
    const int ric = has ? ri : 0;
    int slot = S.ref_slot[min(slice, INTER4_LDS_SLICES - 1)][l][ric];
    if (slice >= INTER4_LDS_SLICES)
        slot = (int8_t)slice_byte(slices, slice, (int)offsetof(h264r_slice, ref_slot) + l * H264R_MAX_REFS + ric);
    slot = has ? slot : -1;
    return make_uint2(mv, (uint32_t)(uint8_t)ri | ((uint32_t)(uint8_t)slot << 8));
}
DEV uint2 block_motion(const h264r_batch& b, const h264r_slice* slices, const Inter4Lds& S, size_t at, int slice, int l)
{
    return motion_word(b.mv[at], b.ref_idx[at], slices, S, slice, l);
}

DEV h264r_mb mb_lane(const h264r_mb* p)          // per-lane 32-byte record, two 16-byte loads
{
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 w0 = q[0], w1 = q[1];
    h264r_mb m;
    uint32_t* w = reinterpret_cast<uint32_t*>(&m);
    w[0] = w0.x; w[1] = w0.y; w[2] = w0.z; w[3] = w0.w; w[4] = w1.x; w[5] = w1.y; w[6] = w1.z; w[7] = w1.w;
    return m;
}

// A lane's MB record, its block's motion ({mv, ref_idx} per list) and the slice header:
// none depends on the workgroup's LDS tables, so the kernels issue them before filling
// those tables (one global round trip less in front of the motion compensation).
struct Inter4Pre {
    h264r_mb q;
    uint32_t mv[2];
    int ri[2];
};
DEV Inter4Pre inter4_pre(const h264r_batch& b, const Geom& g, int pic, int a0, int aend, int lane)
{
    const int blk = lane & 15, a = a0 + (lane >> 4);
    const int aa = a < aend ? a : aend - 1;
    const int mbx = aa % g.wmb, mby = aa / g.wmb;
    const int mi = (mby * 4 + (blk >> 2)) * g.W4 + mbx * 4 + (blk & 3);
    const size_t mbase = (size_t)pic * 2 * g.motion_plane;
    Inter4Pre p;
    p.q = mb_lane(&b.mbs[(size_t)pic * g.nmb + aa]);
#pragma unroll
    for (int l = 0; l < 2; ++l) {
        p.mv[l] = b.mv[mbase + l * g.motion_plane + mi];
        p.ri[l] = b.ref_idx[mbase + l * g.motion_plane + mi];
    }
    return p;
}

// What the deblocking record of a lane's block reads besides its own MB: the left and upper
// MB records and the motion of the blocks left of and above it (the MB's own blocks or the
// neighbours'), loaded unconditionally and with no dependence on the MB record, so k_inter4r
// issues them together with inter4_pre's loads (one global round trip per group).
struct DbNb {
    h264r_mb L, U;
    uint32_t lmv[2], umv[2];
    int lri[2], uri[2];
};
DEV DbNb dbinfo_pre(const h264r_batch& b, const Geom& g, int pic, int a0, int aend, int lane)
{
    const int blk = lane & 15, a = a0 + (lane >> 4);
    const int aa = a < aend ? a : aend - 1;
    const int mbx = aa % g.wmb, mby = aa / g.wmb;
    const int X4 = mbx * 4 + (blk & 3), Y4 = mby * 4 + (blk >> 2);
    const int mi = Y4 * g.W4 + X4;
    const int li = X4 > 0 ? mi - 1 : mi, ui = Y4 > 0 ? mi - g.W4 : mi;
    const size_t mbase = (size_t)pic * 2 * g.motion_plane;
    const h264r_mb* mbs = b.mbs + (size_t)pic * g.nmb;
    DbNb n;
    n.L = mb_lane(&mbs[mbx > 0 ? aa - 1 : aa]);
    n.U = mb_lane(&mbs[mby > 0 ? aa - g.wmb : aa]);
#pragma unroll
    for (int l = 0; l < 2; ++l) {
        n.lmv[l] = b.mv[mbase + l * g.motion_plane + li];
        n.lri[l] = b.ref_idx[mbase + l * g.motion_plane + li];
        n.umv[l] = b.mv[mbase + l * g.motion_plane + ui];
        n.uri[l] = b.ref_idx[mbase + l * g.motion_plane + ui];
    }
    return n;
}

DEV int sel16(uint32_t lo, uint32_t hi, int c) { return (int16_t)(((c & 2) ? hi : lo) >> (16 * (c & 1))); }

// ---------------------------------------------------------------- packed 16-bit helpers
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
DEV s16x2 as_s16x2(uint32_t v) { return __builtin_bit_cast(s16x2, v); }
DEV uint32_t as_u32(s16x2 v) { return __builtin_bit_cast(uint32_t, v); }
DEV s16x2 splat16(short v) { return (s16x2){v, v}; }
DEV s16x2 pk_max(s16x2 a, s16x2 b) { return __builtin_elementwise_max(a, b); }
DEV s16x2 pk_min(s16x2 a, s16x2 b) { return __builtin_elementwise_min(a, b); }
DEV s16x2 pk_clip255(s16x2 a) { return pk_min(pk_max(a, splat16(0)), splat16(255)); }
// (p[k], p[k+1]) of the 9 row samples held as bytes in r0 = p0..p3, r1 = p4..p7, r2 = p8
template <int K>
DEV s16x2 pair_at(uint32_t r0, uint32_t r1, uint32_t r2)
{
    constexpr uint32_t sel = K < 3 ? (0x0c000c00u | ((K + 1) << 16) | K)
                           : K == 3 ? 0x0c040c03u
                           : K < 7 ? (0x0c000c00u | ((K - 3) << 16) | (K - 4))
                           : 0x0c040c03u;
    return as_s16x2(K < 4 ? __builtin_amdgcn_perm(r1, r0, sel) : __builtin_amdgcn_perm(r2, r1, sel));
}

// The 16 luma prediction samples of one 4x4 block at integer position (x, y) and
// quarter phase (xf, yf): spec 8.4.2.2.1 / reference get_block_luma
// (inter_prediction.cc:158-340).  The 9 window rows y-2..y+6 are loaded at once and
// streamed; per row the unrounded horizontal 6-tap b1 of columns 0..3 is computed
// once (packed 16-bit pairs, exact: |b1| <= 10710) and feeds both b (rows 2..6) and
// the centre j of every output row it is a tap of (32-bit); the vertical 6-tap h of
// column c + 2 (+1 for xf == 3: m) accumulates in packed 16-bit.  Every output is
// (X + Y + 1) >> 1 of two of {G, b, h, j}, chosen per lane from the phase.
// out[i] packs row i's four samples as bytes.
// The 9 window rows of one lane straight from the reference plane (three aligned dwords
// per row from clip(x - 2) & ~3, row index clamped).
DEV void luma_window_global(const uint8_t* __restrict__ img, int W, int pitch, int H, int x, int y, uint32_t (&w)[9][3])
{
#pragma unroll
    for (int r = 0; r < 9; ++r) {
        const gdword* q = row_dwords(img, W, pitch, H, x, y - 2 + r);
        w[r][0] = q[0]; w[r][1] = q[1]; w[r][2] = q[2];
    }
}

// (The LDS reference-tile variant of round 3 -- one 13-row tile per 8x8 quadrant by LDS-DMA,
// measured slower, profiles/r03_e_ab.txt -- is gone, and since round 5 so is its never-taken
// branch, which had steered k_inter4r's register allocation: each output row is finished as
// soon as its last tap row is in, so its accumulators are free for the rest of the window and
// the kernel fits 128 VGPRs without it.)
DEV void luma_block_pred(const uint32_t (&w)[9][3], int W, int x, int xf, int yf, uint32_t (&out)[4])
{
    const int hs = xf == 3 ? 1 : 0;                  // G / h column c + 2 + hs
    const int brow = yf == 3 ? 1 : 0;                // b / G row i + 2 + brow
    const bool inside = x - 2 >= 0 && x + 6 < W;
    const int sh = (x - 2) & 3;
    // output = (X + Y + 1) >> 1, X, Y in {0 G, 1 b, 2 h, 3 j}: (xs, ys) of the 16 phases as a
    // 64-bit table (an if-chain on the lane's phase compiled to lane-divergent branches)
    // XSYS nibble 4 xf + yf = xs | ys << 2:  xf 0: (0,0) (0,2) (2,2) (0,2); yf 0: (0,1) (1,1)
    // (0,1); xf 2: (1,3) (3,3) (1,3); yf 2: (2,3); else (1,2)
    constexpr uint64_t XSYS = 0x9e94dfd59e948a80ull;
    const int xsys = (int)(XSYS >> (4 * (xf * 4 + yf))) & 15, xs = xsys & 3, ys = xsys >> 2;
    // one of four by masks (a ternary chain became a branch tree)
    const uint32_t mx1 = 0u - (uint32_t)(xs & 1), mx2 = 0u - (uint32_t)(xs >> 1);
    const uint32_t my1 = 0u - (uint32_t)(ys & 1), my2 = 0u - (uint32_t)(ys >> 1);
    auto pick = [](uint32_t m1, uint32_t m2, uint32_t a, uint32_t b, uint32_t c, uint32_t d) -> uint32_t {
        const uint32_t lo = a ^ ((a ^ b) & m1), hi = c ^ ((c ^ d) & m1);
        return lo ^ ((lo ^ hi) & m2);
    };
    s16x2 hacc[4][2], bsv[4][2], gsv[4][2];
    // the centre j's vertical 6-tap over b1 (|sum| < 2^20) in packed fp32, exact below 2^24:
    // two columns per v_pk_fma_f32 instead of one 32-bit multiply-add each
    f32x2 jacc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
            hacc[i][h2] = bsv[i][h2] = gsv[i][h2] = splat16(0);
            jacc[i][h2] = (f32x2){0.f, 0.f};
        }
    }
    constexpr short C6[6] = {1, -5, 20, 20, -5, 1};
#pragma unroll
    for (int r = 0; r < 9; ++r) {
        uint32_t r0, r1, r2;
        if (inside) {
            r0 = __builtin_amdgcn_alignbyte(w[r][1], w[r][0], sh);
            r1 = __builtin_amdgcn_alignbyte(w[r][2], w[r][1], sh);
            r2 = w[r][2] >> (8 * sh);
        } else {                                       // window crosses the picture edge: clamp per sample
            int p[9];
            row9(w[r][0], w[r][1], w[r][2], x, W, p);
            r0 = p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24);
            r1 = p[4] | (p[5] << 8) | (p[6] << 16) | ((uint32_t)p[7] << 24);
            r2 = p[8];
        }
        const s16x2 q0 = pair_at<0>(r0, r1, r2), q1 = pair_at<1>(r0, r1, r2), q2 = pair_at<2>(r0, r1, r2);
        const s16x2 q3 = pair_at<3>(r0, r1, r2), q4 = pair_at<4>(r0, r1, r2), q5 = pair_at<5>(r0, r1, r2);
        const s16x2 q6 = pair_at<6>(r0, r1, r2), q7 = pair_at<7>(r0, r1, r2);
        const s16x2 b01 = (q0 + q5) + splat16(20) * (q2 + q3) - splat16(5) * (q1 + q4);   // b1 cols 0,1
        const s16x2 b23 = (q2 + q7) + splat16(20) * (q4 + q5) - splat16(5) * (q3 + q6);   // b1 cols 2,3
        const s16x2 g01 = hs ? q3 : q2, g23 = hs ? q5 : q4;                                // G column pairs
        const f32x2 bf[2] = {(f32x2){(float)b01.x, (float)b01.y}, (f32x2){(float)b23.x, (float)b23.y}};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = r - i;                       // tap index of row r for output row i
            if (k < 0 || k > 5) continue;
            hacc[i][0] += splat16(C6[k]) * g01;
            hacc[i][1] += splat16(C6[k]) * g23;
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2)
                jacc[i][h2] = __builtin_elementwise_fma((f32x2){(float)C6[k], (float)C6[k]}, bf[h2], jacc[i][h2]);
            if (k == 2 || k == 3) {                    // b / G of output row i: row i + 2 + brow
                const bool take = k == 2 + brow;
                bsv[i][0] = take ? b01 : bsv[i][0];
                bsv[i][1] = take ? b23 : bsv[i][1];
                gsv[i][0] = take ? g01 : gsv[i][0];
                gsv[i][1] = take ? g23 : gsv[i][1];
            }
        }
        // output row i has all its taps after row i + 5: finished here, its accumulators free
        if (r >= 5) {
            const int i = r - 5;
            uint32_t o2[2];
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2) {
                const s16x2 G = gsv[i][h2];
                const s16x2 hh = pk_clip255((hacc[i][h2] + splat16(16)) >> splat16(5));
                const s16x2 bb = pk_clip255((bsv[i][h2] + splat16(16)) >> splat16(5));
                // (j1 + 512) >> 10 clipped: j1 / 1024 + 0.5 is exact, and truncation equals the
                // floor wherever the clip does not send the value to 0 anyway
                const f32x2 jf = __builtin_elementwise_fma(jacc[i][h2], (f32x2){1.f / 1024.f, 1.f / 1024.f}, (f32x2){0.5f, 0.5f});
                const int j0 = (int)__builtin_amdgcn_fmed3f(jf.x, 0.f, 255.f), j1 = (int)__builtin_amdgcn_fmed3f(jf.y, 0.f, 255.f);
                // all four computed, then picked per lane (the phase differs between lanes)
                const uint32_t g32 = as_u32(G), b32 = as_u32(bb), h32 = as_u32(hh), j32 = (uint32_t)j0 | ((uint32_t)j1 << 16);
                const s16x2 X = as_s16x2(pick(mx1, mx2, g32, b32, h32, j32));
                const s16x2 Y = as_s16x2(pick(my1, my2, g32, b32, h32, j32));
                o2[h2] = as_u32((X + Y + splat16(1)) >> splat16(1));
            }
            out[i] = __builtin_amdgcn_perm(o2[1], o2[0], 0x06040200u);
        }
    }
}

// 2x2 chroma prediction samples at chroma integer position (xi, yi), eighth phase
// (xf, yf): get_block_chroma inter_prediction.cc:380-404 with clamped coordinates.
// Both planes; each plane's four samples as bytes (row 0 in bits 0..15, row 1 in 16..31).
// A row's three clamped samples come out of its two dwords by one byte permute (the
// selector computed once per lane), and the two samples of an output row are one packed
// 16-bit sum: (8-xf)(8-yf) + xf(8-yf) + (8-xf)yf + xf yf = 64, so 255 * 64 + 32 fits.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
DEV u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
DEV void chroma_block_pred2(const uint8_t* __restrict__ cb, const uint8_t* __restrict__ cr, int W, int pitch, int H, int xi,
                            int yi, int xf, int yf, uint32_t (&out)[2])
{
    const int a = clip3(0, W - 1, xi) & ~3;
    // both planes' three rows first (12 dwords in flight): a lane-divergent interior / edge
    // split made every row's load wait for the previous row's use, and one plane at a time
    // left the second plane's last row behind a full vmcnt wait
    uint32_t w[2][3][2];
#pragma unroll
    for (int pl = 0; pl < 2; ++pl)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const gdword* q = as_global((pl ? cr : cb) + (size_t)clip3(0, H - 1, yi + k) * pitch + a);
            w[pl][k][0] = q[0];
            w[pl][k][1] = q[1];
        }
    // byte c (c = 0..2) of the selector: the clamped column's byte in {dword 0 (0..3), dword 1
    // (4..7)}; byte 3 reads zero
    uint32_t sel = 0x0c000000u;
#pragma unroll
    for (int c = 0; c < 3; ++c) sel |= (uint32_t)(clip3(0, W - 1, xi + c) - a) << (8 * c);
    const u16x2 wa = (u16x2)(unsigned short)((8 - xf) * (8 - yf)), wb = (u16x2)(unsigned short)(xf * (8 - yf));
    const u16x2 wc = (u16x2)(unsigned short)((8 - xf) * yf), wd = (u16x2)(unsigned short)(xf * yf);
#pragma unroll
    for (int pl = 0; pl < 2; ++pl) {
        u16x2 A[3], B[3];                       // row k: {p[k][0], p[k][1]} and {p[k][1], p[k][2]}
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint32_t r = __builtin_amdgcn_perm(w[pl][k][1], w[pl][k][0], sel);
            A[k] = as_u16x2(__builtin_amdgcn_perm(r, r, 0x0c010c00u));
            B[k] = as_u16x2(__builtin_amdgcn_perm(r, r, 0x0c020c01u));
        }
        uint32_t o[2];
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            const u16x2 v = (wa * A[rr] + wb * B[rr] + wc * A[rr + 1] + wd * B[rr + 1] + (u16x2)(unsigned short)32) >> (u16x2)(unsigned short)6;
            o[rr] = __builtin_bit_cast(uint32_t, v);
        }
        out[pl] = __builtin_amdgcn_perm(o[1], o[0], 0x06040200u);
    }
}

// mc_prediction / bi_prediction combine (inter_prediction.cc:53-156) of one lane and
// plane as w0 * v0 + w1 * v1, rounded right shift by d (rshift_rnd :35-38), + o, with the
// reference's case split resolved once per plane instead of per sample: one list unweighted
// {1, 0 | 0, 1; d 0}, one list explicit {w, 0 | 0, w; logWD; o}, both lists unweighted
// {1, 1; 1}, explicit {w0, w1; logWD + 1; (o0 + o1 + 1) >> 1}, implicit {64 - w1, w1;
// logWD + 1 = 6}.  The slice's weights are loaded together, not per sample behind branches.
struct WpPar {
    int w0, w1, o, d, rnd;
};
// The slice's weights and offsets of both lists' references, all three planes, loaded
// together (per-plane loads behind the case split below waited for each other: three round
// trips per MB in weighted slices)
struct WpRaw {
    int lwd[2];
    int wa[3], wb[3], oa[3], ob[3];
    int iw;
};
DEV WpRaw wp_raw(const h264r_slice* __restrict__ sl, int r0, int r1)
{
    const int ra = clip3(0, H264R_MAX_REFS - 1, r0), rb = clip3(0, H264R_MAX_REFS - 1, r1);   // unused list: any entry
    WpRaw w;
    w.lwd[0] = sl->luma_log2_wd;
    w.lwd[1] = sl->chroma_log2_wd;
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
        w.wa[pl] = sl->wp_weight[0][ra][pl];
        w.wb[pl] = sl->wp_weight[1][rb][pl];
        w.oa[pl] = sl->wp_offset[0][ra][pl];
        w.ob[pl] = sl->wp_offset[1][rb][pl];
    }
    w.iw = sl->implicit_w1[ra][rb];
    return w;
}
DEV WpPar wp_params(const WpRaw& w, int wp_mode, int dir, int pl)
{
    const int lwd = w.lwd[pl ? 1 : 0];
    const int wa = w.wa[pl], wb = w.wb[pl], oa = w.oa[pl], ob = w.ob[pl], iw = w.iw;
    // selects, not branches (dir and the slice's mode differ between a wave's lanes): one
    // list (explicit weights or plain), both lists averaged, explicit or implicit
    WpPar p;
    const bool ex = wp_mode == 1, im = wp_mode == 2, bi = dir == 2;
    p.w0 = bi ? (ex ? wa : (im ? 64 - iw : 1)) : (dir == 0 ? (ex ? wa : 1) : 0);
    p.w1 = bi ? (ex ? wb : (im ? iw : 1)) : (dir == 1 ? (ex ? wb : 1) : 0);
    p.o = bi ? (ex ? (oa + ob + 1) >> 1 : 0) : (ex ? (dir == 0 ? oa : ob) : 0);
    p.d = bi ? (wp_mode == 0 ? 1 : lwd + 1) : (ex ? lwd : 0);
    p.rnd = p.d > 0 ? 1 << (p.d - 1) : 0;
    return p;
}
// 4 packed samples of each list
DEV uint32_t wp_apply4(const WpPar& p, uint32_t v0, uint32_t v1)
{
    uint32_t o = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int x = p.w0 * (int)((v0 >> (8 * c)) & 255) + p.w1 * (int)((v1 >> (8 * c)) & 255);
        o |= (uint32_t)clip255(((x + p.rnd) >> p.d) + p.o) << (8 * c);
    }
    return o;
}
// The combine of 4 packed samples: weighted prediction off is byte-wise SWAR.
DEV uint32_t wp_combine4(const WpPar& p, int wp_mode, int dir, uint32_t v0, uint32_t v1)
{
    if (wp_mode == 0) {
        // one list or (a + b + 1) >> 1 per byte, selected (dir differs between a wave's lanes)
        const uint32_t avg = (v0 | v1) - (((v0 ^ v1) >> 1) & 0x7F7F7F7Fu);
        return dir == 0 ? v0 : (dir == 1 ? v1 : avg);
    }
    return wp_apply4(p, v0, v1);
}

// 4-point inverse transform of one column / row held in registers, (x + 32) >> 6 at
// the end of the second pass (inverse_4x4 transform.cc:597-641).
DEV void idct4_inplace(int& a, int& b, int& c, int& d)
{
    int o0, o1, o2, o3;
    idct4(a, b, c, d, o0, o1, o2, o3);
    a = o0; b = o1; c = o2; d = o3;
}

// ------------------------------------------------------------------ SP slices
// Transform::itrans_sp / itrans_sp_cr (transform.cc:1098-1265), the arithmetic of the
// reference as it stands (see oracle/h264r_oracle.c sp_mb for its quirks).
__device__ static const uint8_t SP_A[16] = {16, 20, 16, 20, 20, 25, 20, 25, 16, 20, 16, 20, 20, 25, 20, 25};
DEV int sp_sgn(int x) { return (x >= 0) - (x < 0); }                                   // defines.h:73-77
DEV int sp_ls2(int m, int j, int i)                                                     // LevelScale2 :1105-1130
{
    const int cls = (j & 1) + (i & 1);
    constexpr int v0[6] = {13107, 11916, 10082, 9362, 8192, 7282};
    constexpr int v1[6] = {8066, 7490, 6554, 5825, 5243, 4559};
    constexpr int v2[6] = {5243, 4660, 4194, 3647, 3355, 2893};
    return cls == 0 ? v0[m] : (cls == 1 ? v1[m] : v2[m]);
}
DEV int sp_dq(int m, int j, int i)                                                      // dequant_coef :93-100
{
    constexpr int v0[6] = {10, 11, 13, 14, 16, 18};
    constexpr int v1[6] = {13, 14, 16, 18, 20, 23};
    constexpr int v2[6] = {16, 18, 20, 23, 25, 29};
    const int cls = (j & 1) + (i & 1);
    return cls == 0 ? v0[m] : (cls == 1 ? v1[m] : v2[m]);
}
// One coefficient of itrans_sp (luma, :1158-1178): cr the dequantised level, cp the
// transformed prediction; returns the re-dequantised coefficient.
DEV int sp_luma_coef(int cr, int cp, int j, int i, int qp, int qs, int sw)
{
    const int ls = sp_ls2(qs % 6, j, i);
    int cij;
    if (sw) {
        cij = cr + sp_sgn(cp) * ((iabs(cp) * ls + (1 << (14 + qs / 6))) >> (15 + qs / 6));
    } else {
        const int cs = cp + ((int)((unsigned)(cr * sp_dq(qp % 6, j, i) * SP_A[j * 4 + i]) << (qp / 6)) >> 10);
        cij = sp_sgn(cs) * ((iabs(cs) * ls + (1 << (14 + qs / 6))) >> (15 + qs / 6));
    }
    const int dq = sp_dq(qs % 6, j, i);
    return qs >= 24 ? (int)((unsigned)(cij * dq) << (qs / 6 - 4)) : (cij * dq + (1 << (3 - qs / 6))) >> (4 - qs / 6);
}
// 4-point forward core transform (forward_4x4 rows / columns, :560-594)
DEV void fwd4(int p0, int p1, int p2, int p3, int& c0, int& c1, int& c2, int& c3)
{
    const int e0 = p0 + p3, e1 = p1 + p2, e2 = p1 - p2, e3 = p0 - p3;
    c0 = e0 + e1; c1 = e2 + (e3 << 1); c2 = e0 - e1; c3 = e3 - (e2 << 1);
}

// QpY (pl 0) / QpC[pl - 1] of a record, from its dwords 0 and 1
DEV int mb_qp(const h264r_mb& m, int pl)
{
    const uint32_t w0 = reinterpret_cast<const uint32_t*>(&m)[0], w1 = reinterpret_cast<const uint32_t*>(&m)[1];
    return pl == 0 ? (int)(int8_t)(w0 >> 24) : (int)(int8_t)(w1 >> (8 * (pl - 1)));
}

// The deblocking record of one MB's 4x4 block (Deblock::strength deblock.cc:78-289,
// edge parameters :469-480): the block's left edge (vertical edge bx, segment by) and top
// edge (horizontal edge by, segment bx), and for blk < 9 one alpha/beta/tc0 word.  Inside
// k_inter4r, before the group's reconstruction.
DEV void dbinfo_block(const h264r_batch& b, const Geom& g, int pic, int aa, bool valid, int blk, const Inter4Lds& S, const DbTables& T,
                      const h264r_mb& q, uint2 m0, uint2 m1, uint2 qsh, const DbNb& nb, DbInfo* __restrict__ dbout)
{
    const int bx = blk & 3, by = blk >> 2;
    const int mbx = aa % g.wmb, mby = aa / g.wmb;
    const h264r_slice* slices = b.slices + (size_t)pic * b.slice_stride;
    const int hasL = mbx > 0, hasU = mby > 0;
    const int q_type = qsh.x & 255, idc = (qsh.x >> 8) & 255;
    const int offa = (int8_t)((qsh.x >> 16) & 255), offb = (int8_t)(qsh.x >> 24);
    const h264r_mb& L = nb.L;
    const h264r_mb& U = nb.U;
    // the neighbour block belongs to this MB or to the left / upper one (its slice resolves it)
    const int lsl = bx > 0 ? q.slice : L.slice, usl = by > 0 ? q.slice : U.slice;
    const uint2 l0 = motion_word(nb.lmv[0], nb.lri[0], slices, S, lsl, 0), l1 = motion_word(nb.lmv[1], nb.lri[1], slices, S, lsl, 1);
    const uint2 u0 = motion_word(nb.umv[0], nb.uri[0], slices, S, usl, 0), u1 = motion_word(nb.umv[1], nb.uri[1], slices, S, usl, 1);
    const int l_type = slice_type_of(slices, S, L.slice), u_type = slice_type_of(slices, S, U.slice);
    // field pictures: mvlimit 2 (deblock.cc:86,164) and no bS 4 across horizontal MB edges
    // (cond_bS4 = !field || vertical, deblock.cc:103-107,184-189)
    const int fld = (int)__builtin_amdgcn_readfirstlane(ld_const(&b.pics[pic].structure)) != H264R_FRAME;
    const int mvlim = fld ? 2 : 4;
    // ---- deblocking record (Deblock::strength deblock.cc:78-289): this lane's
    // left edge (vertical edge bx, segment by) and top edge (horizontal edge by,
    // segment bx)
    if (valid) {
        const int fl = idc == 0 ? hasL : (idc == 2 && hasL && L.slice == q.slice);
        const int ft = idc == 0 ? hasU : (idc == 2 && hasU && U.slice == q.slice);
        const int t8 = (q.flags & H264R_MBF_T8x8) != 0;
        const MotionRef mq = motion_of(m0, m1);
        const int q_intra = mb_is_intra(q);
        const int pskip = q_type == H264R_SLICE_P && q.mb_type == H264R_P_SKIP;
        const int special_q = special_slice(q_type);
        DbInfo* out = dbout + aa;
#pragma unroll
        for (int hor = 0; hor < 2; ++hor) {
            const int e = hor ? by : bx, s = hor ? bx : by;
            const int en = idc != 1 && (e == 0 ? (hor ? ft : fl) : ((e & 1) ? !t8 : 1));
            int v = 0;
            if (en) {
                // MB P of the edge: the left / upper MB for edge 0, else this MB
                const int p_flags = e == 0 ? (hor ? U.flags : L.flags) : q.flags;
                const int p_cbp = e == 0 ? (hor ? U.cbp_blks : L.cbp_blks) : q.cbp_blks;
                const int special = special_q || (e == 0 && special_slice(hor ? u_type : l_type));
                const int intra = q_intra || (p_flags & H264R_MBF_INTRA) != 0;
                const int blkQ = 4 * by + bx;
                const int blkP = hor ? (e == 0 ? 12 + bx : blkQ - 4) : (e == 0 ? blkQ + 3 : blkQ - 1);
                const int coded = ((q.cbp_blks >> blkQ) & 1) || ((p_cbp >> blkP) & 1);
                const int same_part = e > 0 && (q.mb_type == H264R_P_16x16 ||
                                                q.mb_type == (hor ? H264R_P_8x16 : H264R_P_16x8));
                if (!hor) {
                    if (special) v = e == 0 ? 4 : 3;
                    else if (e > 0 && pskip) v = 0;
                    else if (e == 0 && intra) v = 4;
                    else if (intra) v = 3;
                    else if (coded) v = 2;
                    else if (same_part) v = 0;
                    else v = bs_compare(mq, motion_of(l0, l1), mvlim);
                } else {
                    if (e == 0 && !fld && (special || intra)) v = 4;
                    else if (special || intra) v = 3;
                    else if (e > 0 && pskip) v = 0;
                    else if (coded) v = 2;
                    else if (same_part) v = 0;
                    else v = bs_compare(mq, motion_of(u0, u1), mvlim);
                }
            }
            out->bs[hor * 16 + e * 4 + s] = (uint8_t)v;
        }
        if (blk < 9) {                                              // edge parameters
            const int pl = blk / 3, which = blk - pl * 3;
            // QP of plane pl from the record's dwords 0 / 1 (a select between the byte fields
            // became a select of their addresses: the record went to memory, promoted to LDS)
            const h264r_mb& P = which == 0 ? L : (which == 1 ? U : q);
            const int qp = mb_qp(P, pl), qq = mb_qp(q, pl);
            out->par[blk] = edge_word(qp, qq, offa, offb, T.ab, T.tc0);
        }
    }
}

// The inter / I_PCM macroblocks a0 .. a0+3 of picture `pic` (their deblocking records come
// first, dbinfo_block).  SP = false (k_inter4r): inter MBs of SP slices are left out and flagged in
// *sp_flag (the launch tag); SP = true (k_inter_sp): only those are reconstructed, with inverse_transform_sp
// (decoder.cc:256-257, transform.cc:1267-1300).
template <bool SP>
DEV void inter4_mbs(const h264r_batch& b, const Geom& g, int pic, int a0, int aend, int lane,
                    const Inter4Lds& S, int* sp_flag, const Inter4Pre& pre, uint8_t* __restrict__ recon, int tag)
{
    const int grp = lane >> 4, blk = lane & 15, bx = blk & 3, by = blk >> 2;
    const int a = a0 + grp;
    const bool valid = a < aend;
    const int aa = valid ? a : aend - 1;
    const int mbx = aa % g.wmb, mby = aa / g.wmb;
    const h264r_slice* slices = b.slices + (size_t)pic * b.slice_stride;

    // ---- MB record (inter4_pre: two 16-byte loads -- a struct copy becomes one byte load
    // per field, each waited on its own) and the motion of this block
    const int X4 = mbx * 4 + bx, Y4 = mby * 4 + by;
    const h264r_mb q = pre.q;
    const h264r_slice* qs = &slices[q.slice];
    const uint2 qsh = slice_hdr(slices, S, q.slice);
    const uint2 m0 = motion_word(pre.mv[0], pre.ri[0], slices, S, q.slice, 0);
    const uint2 m1 = motion_word(pre.mv[1], pre.ri[1], slices, S, q.slice, 1);
    const int q_type = qsh.x & 255;
    const int wp_mode = qsh.y & 255;

    // ---- reconstruction of inter / I_PCM MBs (intra MBs: the lanes idle here)
    [&]() {
        const bool pcm = q.mb_type == H264R_I_PCM;
        if (!valid || (mb_is_intra(q) && !pcm)) return;              // intra: k_intra_* (lanes idle here)
        const bool sp_mb = q_type == H264R_SLICE_SP && !mb_is_intra(q);
        if constexpr (!SP) {
            if (sp_mb) { *sp_flag = tag; return; }                   // k_inter_sp's
        } else {
            if (!sp_mb) return;
        }
        const int16_t* lv = b.levels + q.coef_off;
        // my 4x4 block in the MB-tiled reconstruction (device_common.h): rows of 16 / 8 bytes
        uint8_t* const rmb = recon_mb(recon, g, pic, aa);
        uint8_t* ydst = rmb + (by * 4) * 16 + bx * 4;
        const int coff = RECON_CB + (by * 2) * 8 + bx * 2;          // Cb; Cr 64 bytes on
        if (pcm) {                                                       // mb_pred_ipcm decoder.cc:149-168
            const uint8_t* raw = reinterpret_cast<const uint8_t*>(lv);
    #pragma unroll
            for (int r = 0; r < 4; ++r)
                *reinterpret_cast<uint32_t*>(ydst + r * 16) =
                    *reinterpret_cast<const uint32_t*>(raw + (by * 4 + r) * 16 + bx * 4);
    #pragma unroll
            for (int pl = 0; pl < 2; ++pl)
    #pragma unroll
                for (int r = 0; r < 2; ++r)
                    *reinterpret_cast<uint16_t*>(rmb + coff + pl * 64 + r * 8) =
                        *reinterpret_cast<const uint16_t*>(raw + 256 + pl * 64 + (by * 2 + r) * 8 + bx * 2);
            return;
        }

        // ---- residual inputs: issued after the motion compensation, so that they are not
        // live across it (30 VGPRs: k_inter4r fits 128 VGPRs = 4 waves/SIMD; config 3
        // 475 -> 493 M MB/s, profiles/r03_h_inter_ab.txt)
        const int cbpl = q.cbp & 15, cbpc = q.cbp >> 4;
        const int t8 = (q.flags & H264R_MBF_T8x8) != 0;
        const h264r_quant* __restrict__ qt = &b.quant[pic];
        const int qpl = q.qp_scaled[0];
        const int b8 = (by >> 1) * 2 + (bx >> 1);
        const int loff = b8_offset(q.cbp, b8);
        uint4 lev[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
        uint4 lsc[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
        // chroma: my 2x2 quadrant of chroma 4x4 block cb of each plane + the plane's 4 DC levels
        const int cb = (by >> 1) * 2 + (bx >> 1), cr = (by & 1) * 2, cc = (bx & 1) * 2;
        uint32_t clev[2][2] = {{0, 0}, {0, 0}}, csc[2][2] = {{0, 0}, {0, 0}};
        uint2 cdc[2] = {make_uint2(0, 0), make_uint2(0, 0)};
        int cdcs[2] = {0, 0};
        auto load_residual = [&]() {
            if (loff >= 0) {
                if (!t8) {                      // 4x4 block: 16 raster levels
                    const uint4* p = reinterpret_cast<const uint4*>(lv + loff + ((by & 1) * 2 + (bx & 1)) * 16);
                    lev[0] = p[0]; lev[1] = p[1];
                    const uint4* s = reinterpret_cast<const uint4*>(&qt->scale4x4[1][0][qpl % 6][0]);
                    lsc[0] = s[0]; lsc[1] = s[1];
                } else {                        // my 4x4 quadrant of the 8x8 block: rows (by&1)*4.., cols (bx&1)*4..
                    const int16_t* p = lv + loff + (by & 1) * 32 + (bx & 1) * 4;
                    const int16_t* s = &qt->scale8x8[1][0][qpl % 6][(by & 1) * 32 + (bx & 1) * 4];
                    const uint2 r0 = ld8(p), r1 = ld8(p + 8), r2 = ld8(p + 16), r3 = ld8(p + 24);
                    lev[0] = make_uint4(r0.x, r0.y, r1.x, r1.y); lev[1] = make_uint4(r2.x, r2.y, r3.x, r3.y);
                    const uint2 s0 = ld8(s), s1 = ld8(s + 8), s2 = ld8(s + 16), s3 = ld8(s + 24);
                    lsc[0] = make_uint4(s0.x, s0.y, s1.x, s1.y); lsc[1] = make_uint4(s2.x, s2.y, s3.x, s3.y);
                }
            }
            if (cbpc) {
                const LevelOffs lo = level_offsets(q);
    #pragma unroll
                for (int pl = 0; pl < 2; ++pl) {
                    const int qpc = q.qp_scaled[1 + pl];
                    cdc[pl] = ld8(lv + lo.cdc + pl * 4);
                    cdcs[pl] = qt->scale4x4[1][1 + pl][qpc % 6][0];
                    if (cbpc == 2) {
    #pragma unroll
                        for (int r = 0; r < 2; ++r) {
                            clev[pl][r] = *reinterpret_cast<const uint32_t*>(lv + lo.cac + pl * 64 + cb * 16 + (cr + r) * 4 + cc);
                            csc[pl][r] = *reinterpret_cast<const uint32_t*>(&qt->scale4x4[1][1 + pl][qpc % 6][(cr + r) * 4 + cc]);
                        }
                    }
                }
            }
        };

        // ---- prediction
        const int r0 = (int8_t)(m0.y & 255), r1 = (int8_t)(m1.y & 255);
        const int dir = (r0 >= 0 && r1 >= 0) ? 2 : (r0 >= 0 ? 0 : 1);
        // the prediction of each list in named registers: an array indexed by the (not
        // unrolled) list loop was promoted to LDS by the compiler (48 B per lane)
        uint32_t pY[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, pC[2][2] = {{0, 0}, {0, 0}};
        // a field picture (include/h264r.h H264R_TOP_FIELD) reads fields of the DPB frames:
        // every second row from the field's first row, clamped to the field's own rows
        const int structure = (int)__builtin_amdgcn_readfirstlane(ld_const(&b.pics[pic].structure));
        const int fld = structure != H264R_FRAME;
    #pragma unroll 1
        for (int l = 0; l < 2; ++l) {
            const uint2 mw = l ? m1 : m0;
            const int rr = l ? r1 : r0;
            const bool use = rr >= 0;
            if (!__any(use)) continue;                                  // P pictures: list 1 never
            uint32_t tY[4] = {0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u};
            uint32_t tC[2] = {0x80808080u, 0x80808080u};                // no_ref: 128 (inter_prediction.cc:164-167,366-369)
            const int ref = (int8_t)((mw.y >> 8) & 255);                // slot | H264R_REF_BOTTOM
            const int slot = ref & 31, bot = fld & (ref >> 6);
            const bool ok = use && ref >= 0 && (ref & ~H264R_REF_BOTTOM) < H264R_MAX_SLOTS && rr < H264R_MAX_REFS &&
                            S.planes[slot * 3];
            const int mvx = (int16_t)(mw.x & 0xFFFF), mvy = (int16_t)(mw.x >> 16);
            const int vx = X4 * 16 + mvx, vy = Y4 * 16 + mvy;           // quarter luma / eighth chroma units
            const int x = vx >> 2, y = vy >> 2;
            {
                // the 9 window rows of the lane's own block, straight from the plane
                uint32_t w[9][3];
#if H264R_INTER_DIAG & 4
                // diagnostic build (wrong output): no window loads, no luma filter
                (void)x; (void)y;
                tY[0] = tY[1] = tY[2] = tY[3] = (uint32_t)(vx ^ vy);
#elif H264R_INTER_DIAG & 2
                // diagnostic build (wrong output): the window loads without the luma filter
                if (ok) luma_window_global(S.planes[slot * 3] + bot * g.W, g.W, g.W << fld, g.H, x, y, w);
                if (ok) { uint32_t acc = 0;
    #pragma unroll
                    for (int r = 0; r < 9; ++r) acc ^= w[r][0] ^ w[r][1] ^ w[r][2];
                    tY[0] = tY[1] = tY[2] = tY[3] = acc; }
#else
                if (ok) luma_window_global(S.planes[slot * 3] + bot * g.W, g.W, g.W << fld, g.H, x, y, w);
                if (ok) luma_block_pred(w, g.W, x, vx & 3, vy & 3, tY);
#endif
            }
            // a reference field of the other parity: the chroma sample grid sits a quarter
            // chroma row off (get_block_chroma inter_prediction.cc:352-355)
            const int vyc = vy + (fld && bot != (structure == H264R_BOTTOM_FIELD) ? (bot ? -2 : 2) : 0);
#if H264R_INTER_DIAG & 8
            tC[0] = tC[1] = (uint32_t)vyc;        // diagnostic build (wrong output): no chroma MC
#else
            if (ok) chroma_block_pred2(S.planes[slot * 3 + 1] + bot * g.Wc, S.planes[slot * 3 + 2] + bot * g.Wc, g.Wc,
                                       g.Wc << fld, g.Hc, vx >> 3, vyc >> 3, vx & 7, vyc & 7, tC);
#endif
            const bool l1 = l != 0;
    #pragma unroll
            for (int i = 0; i < 4; ++i) {
                pY[0][i] = (use && !l1) ? tY[i] : pY[0][i];
                pY[1][i] = (use && l1) ? tY[i] : pY[1][i];
            }
    #pragma unroll
            for (int k = 0; k < 2; ++k) {
                pC[0][k] = (use && !l1) ? tC[k] : pC[0][k];
                pC[1][k] = (use && l1) ? tC[k] : pC[1][k];
            }
        }
        uint32_t predY[4], predC[2];
        WpPar wpp[3] = {};
        if (wp_mode != 0) {
            const WpRaw wr = wp_raw(qs, r0, r1);
    #pragma unroll
            for (int pl = 0; pl < 3; ++pl) wpp[pl] = wp_params(wr, wp_mode, dir, pl);
        }
    #pragma unroll
        for (int i = 0; i < 4; ++i) predY[i] = wp_combine4(wpp[0], wp_mode, dir, pY[0][i], pY[1][i]);
    #pragma unroll
        for (int pl = 0; pl < 2; ++pl) predC[pl] = wp_combine4(wpp[1 + pl], wp_mode, dir, pC[0][pl], pC[1][pl]);
#if !(H264R_INTER_DIAG & 16)
        load_residual();
#endif

        if constexpr (SP) {
            // ---- itrans_sp of this lane's 4x4 block (:1132-1187): the prediction is
            // transformed, combined with the level and re-quantised at QsY; the
            // reconstruction is the clipped inverse transform alone
            const int qp = q.qp_y, qsy = qs->qs_y, sw = qs->sp_switch;
            const int per = qpl / 6;
            int cf[4][4];
    #pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int p0 = predY[i] & 255, p1 = (predY[i] >> 8) & 255, p2 = (predY[i] >> 16) & 255, p3 = predY[i] >> 24;
                fwd4(p0, p1, p2, p3, cf[i][0], cf[i][1], cf[i][2], cf[i][3]);
            }
    #pragma unroll
            for (int c = 0; c < 4; ++c) fwd4(cf[0][c], cf[1][c], cf[2][c], cf[3][c], cf[0][c], cf[1][c], cf[2][c], cf[3][c]);
    #pragma unroll
            for (int i = 0; i < 4; ++i)
    #pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const uint4 lw = lev[i >> 1], sw4 = lsc[i >> 1];
                    const uint32_t lo_ = (i & 1) ? lw.z : lw.x, hi_ = (i & 1) ? lw.w : lw.y;
                    const uint32_t slo = (i & 1) ? sw4.z : sw4.x, shi = (i & 1) ? sw4.w : sw4.y;
                    const int cr = dq4(sel16(lo_, hi_, c), sel16(slo, shi, c), per);   // inverse_quantize :409-413
                    cf[i][c] = sp_luma_coef(cr, cf[i][c], i, c, qp, qsy, sw);
                }
    #pragma unroll
            for (int i = 0; i < 4; ++i) idct4_inplace(cf[i][0], cf[i][1], cf[i][2], cf[i][3]);
    #pragma unroll
            for (int c = 0; c < 4; ++c) idct4_inplace(cf[0][c], cf[1][c], cf[2][c], cf[3][c]);
    #pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t wv = 0;
    #pragma unroll
                for (int c = 0; c < 4; ++c) {
                    int v = (cf[i][c] + 32) >> 6;
                    // opaque: shift + clamp + byte packing otherwise becomes v_ashr_pk_u8_i32, whose
                    // upper result half the compiler takes as zero -- on MI355X it kept the old
                    // register's upper bits (bytes 2-3 = 0xFF after a negative input), measured
                    asm volatile("" : "+v"(v));
                    wv |= (uint32_t)clip255(v) << (8 * c);
                }
                *reinterpret_cast<uint32_t*>(ydst + i * 16) = wv;
            }
            // ---- itrans_sp_cr (:1190-1265) then inverse_transform_chroma (:1033-1049):
            // chroma block cb is spread over lanes {blk, ^1, ^4, ^5}; my 2x2 quadrant
            // (rows cr.., cols cc..).  The DC pass takes the raw DC levels (transform_chroma_dc
            // skips SP inter MBs, :865-875), the AC pass the PREDICTION SAMPLES (:1246)
    #pragma unroll
            for (int pl = 0; pl < 2; ++pl) {
                const int qpc = q.qp_c[pl], qsc = qs->qs_c[pl];
                int pr[2][2], f[2][2];
    #pragma unroll
                for (int r = 0; r < 2; ++r)
    #pragma unroll
                    for (int c = 0; c < 2; ++c) pr[r][c] = (predC[pl] >> (16 * r + 8 * c)) & 255;
                // forward transform: rows (my 2 columns + the 2 of lane ^ 1), then columns
                // (my 2 rows + the 2 of lane ^ 4)
                int t[2][2];
    #pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const int o0 = lane_xor1(pr[r][0]), o1 = lane_xor1(pr[r][1]);
                    const int q0 = cc ? o0 : pr[r][0], q1 = cc ? o1 : pr[r][1], q2 = cc ? pr[r][0] : o0, q3 = cc ? pr[r][1] : o1;
                    int y0, y1, y2, y3;
                    fwd4(q0, q1, q2, q3, y0, y1, y2, y3);
                    t[r][0] = cc ? y2 : y0;
                    t[r][1] = cc ? y3 : y1;
                }
    #pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const int o0 = lane_xor4(t[0][c]), o1 = lane_xor4(t[1][c]);
                    const int q0 = cr ? o0 : t[0][c], q1 = cr ? o1 : t[1][c], q2 = cr ? t[0][c] : o0, q3 = cr ? t[1][c] : o1;
                    int y0, y1, y2, y3;
                    fwd4(q0, q1, q2, q3, y0, y1, y2, y3);
                    f[0][c] = cr ? y2 : y0;
                    f[1][c] = cr ? y3 : y1;
                }
                // the four blocks' DC coefficients (lanes 0, 2, 8, 10 of the MB's 16)
                const int gb = lane & ~15;
                const int d00 = __shfl(f[0][0], gb + 0), d01 = __shfl(f[0][0], gb + 2);
                const int d10 = __shfl(f[0][0], gb + 8), d11 = __shfl(f[0][0], gb + 10);
                int mp[4] = {d00 + d10 + d01 + d11, d00 - d10 + d01 - d11, d00 + d10 - d01 - d11, d00 - d10 - d01 + d11};
                const int c00 = (int16_t)(cdc[pl].x & 0xFFFF), c01 = (int16_t)(cdc[pl].x >> 16);
                const int c10 = (int16_t)(cdc[pl].y & 0xFFFF), c11 = (int16_t)(cdc[pl].y >> 16);
                const int crd[4] = {c00, c01, c10, c11};
                const int ls0 = sp_ls2(qsc % 6, 0, 0);
    #pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const int cp = mp[n];
                    int cij;
                    if (qs->sp_switch) {
                        cij = ((sp_sgn(cp) * (iabs(cp) * ls0 + (1 << (15 + qsc / 6)))) >> (16 + qsc / 6)) + cp;
                    } else {
                        const int cs = cp + ((int)((unsigned)(crd[n] * sp_dq(qpc % 6, 0, 0) * 16) << (qpc / 6)) >> 9);
                        cij = (sp_sgn(cs) * (iabs(cs) * ls0 + (1 << (15 + qsc / 6)))) >> (16 + qsc / 6);
                    }
                    mp[n] = (int)((unsigned)(cij * sp_dq(qsc % 6, 0, 0)) << (qpc / 6));
                }
                // AC (every position; (0,0) is replaced by the DC result below)
                int k[2][2];
    #pragma unroll
                for (int r = 0; r < 2; ++r)
    #pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const int j = cr + r, i = cc + c;
                        const int crv = dq4((int16_t)(clev[pl][r] >> (16 * c)), (int16_t)(csc[pl][r] >> (16 * c)), qpc / 6);
                        const int cp = pr[r][c], ls = sp_ls2(qsc % 6, j, i);
                        int cij;
                        if (qs->sp_switch) {
                            cij = crv + ((sp_sgn(cp) * (iabs(cp) * ls + (1 << (14 + qsc / 6)))) >> (15 + qsc / 6));
                        } else {
                            const int cs = cp + ((int)((unsigned)(crv * sp_dq(qpc % 6, j, i) * SP_A[j * 4 + i]) << (qpc / 6)) >> 9);
                            cij = (sp_sgn(cs) * (iabs(cs) * ls + (1 << (14 + qsc / 6)))) >> (15 + qsc / 6);
                        }
                        k[r][c] = (int)((unsigned)(cij * sp_dq(qsc % 6, j, i)) << (qpc / 6));
                    }
                if (cr == 0 && cc == 0) {
                    const int dcv = cb == 0 ? (mp[0] + mp[1] + mp[2] + mp[3]) >> 1
                                  : cb == 1 ? (mp[0] + mp[1] - mp[2] - mp[3]) >> 1
                                  : cb == 2 ? (mp[0] - mp[1] + mp[2] - mp[3]) >> 1
                                            : (mp[0] - mp[1] - mp[2] + mp[3]) >> 1;
                    k[0][0] = dcv;
                }
                // inverse transform (as below) and construction with the prediction
                int rcv[2][2];
                {
                    int tt[2][2];
    #pragma unroll
                    for (int r = 0; r < 2; ++r) {
                        const int o0 = lane_xor1(k[r][0]), o1 = lane_xor1(k[r][1]);
                        const int d0 = cc ? o0 : k[r][0], d1 = cc ? o1 : k[r][1], d2 = cc ? k[r][0] : o0, d3 = cc ? k[r][1] : o1;
                        int y0, y1, y2, y3;
                        idct4(d0, d1, d2, d3, y0, y1, y2, y3);
                        tt[r][0] = cc ? y2 : y0;
                        tt[r][1] = cc ? y3 : y1;
                    }
    #pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const int o0 = lane_xor4(tt[0][c]), o1 = lane_xor4(tt[1][c]);
                        const int d0 = cr ? o0 : tt[0][c], d1 = cr ? o1 : tt[1][c], d2 = cr ? tt[0][c] : o0, d3 = cr ? tt[1][c] : o1;
                        int y0, y1, y2, y3;
                        idct4(d0, d1, d2, d3, y0, y1, y2, y3);
                        rcv[0][c] = ((cr ? y2 : y0) + 32) >> 6;
                        rcv[1][c] = ((cr ? y3 : y1) + 32) >> 6;
                    }
                }
                uint8_t* cdst = rmb + coff + pl * 64;
    #pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const uint32_t wv = (uint32_t)clip255(pr[r][0] + rcv[r][0]) | ((uint32_t)clip255(pr[r][1] + rcv[r][1]) << 8);
                    *reinterpret_cast<uint16_t*>(cdst + r * 8) = (uint16_t)wv;
                }
            }
            return;
        }
        // ---- luma residual (transform.cc:1058-1073)
        int res[4][4];
    #pragma unroll
        for (int i = 0; i < 4; ++i)
    #pragma unroll
            for (int c = 0; c < 4; ++c) res[i][c] = 0;
        const bool byp = (q.flags & H264R_MBF_BYPASS) != 0;
#if H264R_INTER_DIAG & 64
        // diagnostic build (wrong output): the luma levels loaded, not transformed
        res[0][0] = (int)(lev[0].x ^ lev[0].y ^ lev[0].z ^ lev[0].w ^ lev[1].x ^ lev[1].y ^ lev[1].z ^ lev[1].w ^
                          lsc[0].x ^ lsc[1].y) & 3;
#endif
        if (!(H264R_INTER_DIAG & (16 | 64)) && __any(cbpl != 0)) {
            const int per = qpl / 6;
            // dq4 / dq8 (transform.cc:394-419) as one form, rounding and shift per lane: the
            // lanes of a wave mix 4x4 and 8x8 MBs, and a select per value (not a branch) keeps
            // the 16 values free of exec-mask work
            const int drnd = t8 ? 32 : 8, dsh = t8 ? 6 : 4;
            int d[4][4];
    #pragma unroll
            for (int i = 0; i < 4; ++i)
    #pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const uint4 lw = lev[i >> 1], sw = lsc[i >> 1];
                    const uint32_t lo_ = (i & 1) ? lw.z : lw.x, hi_ = (i & 1) ? lw.w : lw.y;
                    const uint32_t slo = (i & 1) ? sw.z : sw.x, shi = (i & 1) ? sw.w : sw.y;
                    const int lvv = sel16(lo_, hi_, c), scv = sel16(slo, shi, c);
                    const int dqv = ((lvv * scv) * (1 << per) + drnd) >> dsh;
                    d[i][c] = byp ? lvv : dqv;
                }
            // lossless MBs (TransformBypassModeFlag): the levels are the residual, DPCM'd in
            // place down the columns / along the rows when the block's Intra4x4PredMode /
            // Intra8x8PredMode is vertical / horizontal (bypass_4x4 / bypass_8x8
            // transform.cc:736-778; inverse_transform_4x4 / _8x8 :986-1016 read those modes
            // for inter MBs too: whatever the parser's mb_t slot holds).  The flag is
            // uniform over an MB's 16 lanes, so the cross-lane carries stay inside the branch.
            if (byp) {
                const uint32_t* qw = reinterpret_cast<const uint32_t*>(&q);
                const uint64_t ipw = (uint64_t)qw[5] | ((uint64_t)qw[6] << 32);
                const int bk = t8 ? b8 : (by >> 1) * 8 + (bx >> 1) * 4 + (by & 1) * 2 + (bx & 1);
                const int mode = (int)((ipw >> (4 * bk)) & 15);
                const bool vert = mode == 0, horz = mode == 1;
    #pragma unroll
                for (int i = 1; i < 4; ++i)
    #pragma unroll
                    for (int c = 0; c < 4; ++c) d[i][c] += vert ? d[i - 1][c] : 0;
    #pragma unroll
                for (int c = 1; c < 4; ++c)
    #pragma unroll
                    for (int i = 0; i < 4; ++i) d[i][c] += horz ? d[i][c - 1] : 0;
                // 8x8: the quadrant above (lane ^ 4) / to the left (lane ^ 1) carries in
    #pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int up = lane_xor4(d[3][c]);
    #pragma unroll
                    for (int i = 0; i < 4; ++i) d[i][c] += (t8 && vert && (by & 1)) ? up : 0;
                }
    #pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int left = lane_xor1(d[i][3]);
    #pragma unroll
                    for (int c = 0; c < 4; ++c) d[i][c] += (t8 && horz && (bx & 1)) ? left : 0;
                }
    #pragma unroll
                for (int i = 0; i < 4; ++i)
    #pragma unroll
                    for (int c = 0; c < 4; ++c) res[i][c] = d[i][c];
            } else
            if (!__any(t8 != 0)) {
                // 4x4: rows then columns, all in-lane
    #pragma unroll
                for (int i = 0; i < 4; ++i) idct4_inplace(d[i][0], d[i][1], d[i][2], d[i][3]);
    #pragma unroll
                for (int c = 0; c < 4; ++c) idct4_inplace(d[0][c], d[1][c], d[2][c], d[3][c]);
    #pragma unroll
                for (int i = 0; i < 4; ++i)
    #pragma unroll
                    for (int c = 0; c < 4; ++c) res[i][c] = (d[i][c] + 32) >> 6;
            } else {
                // 8x8 (only t8 MBs reach here with d != 0 for their lanes; 4x4 MBs of the same
                // wave take the in-lane path below).  Rows: my 4 + the 4 of lane ^ 1.
                int e4[4][4];
    #pragma unroll
                for (int i = 0; i < 4; ++i) {
                    int in[8], outv[8];
    #pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const int ov = lane_xor1(d[i][c]);
                        in[c] = (bx & 1) ? ov : d[i][c];
                        in[4 + c] = (bx & 1) ? d[i][c] : ov;
                    }
                    idct8(in, outv);
                    // mask select: a ternary over the two halves became a lane-indexed array
                    // read, which the compiler placed in LDS (32 B per lane)
                    const int mx = -(bx & 1);
    #pragma unroll
                    for (int c = 0; c < 4; ++c) e4[i][c] = (outv[c] & ~mx) | (outv[4 + c] & mx);
                }
    #pragma unroll
                for (int c = 0; c < 4; ++c) {
                    int in[8], outv[8];
    #pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        in[i] = lane_lo4(e4[i][c]);         // rows 0..3: the lane with by even
                        in[4 + i] = lane_hi4(e4[i][c]);
                    }
                    idct8(in, outv);
                    const int my = -(by & 1);
    #pragma unroll
                    for (int i = 0; i < 4; ++i) res[i][c] = t8 ? ((outv[i] & ~my) | (outv[4 + i] & my)) : 0;
                }
                if (!t8) {
    #pragma unroll
                    for (int i = 0; i < 4; ++i) idct4_inplace(d[i][0], d[i][1], d[i][2], d[i][3]);
    #pragma unroll
                    for (int c = 0; c < 4; ++c) idct4_inplace(d[0][c], d[1][c], d[2][c], d[3][c]);
                }
    #pragma unroll
                for (int i = 0; i < 4; ++i)
    #pragma unroll
                    for (int c = 0; c < 4; ++c) res[i][c] = ((t8 ? res[i][c] : d[i][c]) + 32) >> 6;
            }
        }
        // ---- construction + store, luma
#if H264R_INTER_DIAG & 1
        {   // diagnostic build (wrong output): one 16-byte store per lane, an MB's 16 lanes contiguous
            uint32_t wv4[4];
    #pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t wv = 0;
    #pragma unroll
                for (int c = 0; c < 4; ++c) wv |= (uint32_t)clip255((int)((predY[i] >> (8 * c)) & 255) + res[i][c]) << (8 * c);
                wv4[i] = wv;
            }
            *reinterpret_cast<uint4*>(rmb + blk * 16) = make_uint4(wv4[0], wv4[1], wv4[2], wv4[3]);
        }
#else
    #pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t wv = 0;
    #pragma unroll
            for (int c = 0; c < 4; ++c) wv |= (uint32_t)clip255((int)((predY[i] >> (8 * c)) & 255) + res[i][c]) << (8 * c);
            *reinterpret_cast<uint32_t*>(ydst + i * 16) = wv;
        }
#endif

        // ---- chroma residual (transform.cc:1081-1091, DC :875-889): chroma block cb is
        // spread over lanes {blk, ^1, ^4, ^5}; my quadrant rows cr.., cols cc..
    #pragma unroll
        for (int pl = 0; pl < 2; ++pl) {
            int rc[2][2] = {{0, 0}, {0, 0}};
#if H264R_INTER_DIAG & 128
            // diagnostic build (wrong output): the chroma levels loaded, not transformed
            rc[0][0] = (int)(clev[pl][0] ^ clev[pl][1] ^ csc[pl][0] ^ csc[pl][1] ^ cdc[pl].x ^ cdc[pl].y ^ (uint32_t)cdcs[pl]) & 3;
#endif
            if (!(H264R_INTER_DIAG & (16 | 128)) && __any(cbpc != 0)) {
                const int qpc = q.qp_scaled[1 + pl], per = qpc / 6;
                int k[2][2], raw[2][2];
    #pragma unroll
                for (int r = 0; r < 2; ++r)
    #pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        raw[r][c] = (int16_t)(clev[pl][r] >> (16 * c));
                        k[r][c] = dq4(raw[r][c], (int16_t)(csc[pl][r] >> (16 * c)), per);
                    }
                const int c00 = (int16_t)(cdc[pl].x & 0xFFFF), c01 = (int16_t)(cdc[pl].x >> 16);
                const int c10 = (int16_t)(cdc[pl].y & 0xFFFF), c11 = (int16_t)(cdc[pl].y >> 16);
                const int e00 = c00 + c01, e01 = c00 - c01, e10 = c10 + c11, e11 = c10 - c11;
                // f = (e00 or e01) +/- (e10 or e11) by cb's bits: arithmetic, not a branch tree
                const int ea = (cb & 1) ? e01 : e00, eb = (cb & 1) ? e11 : e10;
                const int f = ea + (eb ^ -(cb >> 1)) + (cb >> 1);
                if (cr == 0 && cc == 0) k[0][0] = cbpc ? ((f * cdcs[pl]) * (1 << per)) >> 5 : 0;
                // rows: my 2 columns + the 2 of lane ^ 1
                int t[2][2];
    #pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const int o0 = lane_xor1(k[r][0]), o1 = lane_xor1(k[r][1]);
                    const int d0 = cc ? o0 : k[r][0], d1 = cc ? o1 : k[r][1], d2 = cc ? k[r][0] : o0, d3 = cc ? k[r][1] : o1;
                    int y0, y1, y2, y3;
                    idct4(d0, d1, d2, d3, y0, y1, y2, y3);
                    t[r][0] = cc ? y2 : y0;
                    t[r][1] = cc ? y3 : y1;
                }
                // columns: my 2 rows + the 2 of lane ^ 4
    #pragma unroll
                for (int c = 0; c < 2; ++c) {
                    // (rows 0..1 from the lane with by even, 2..3 from the other)
                    const int d0 = lane_lo4(t[0][c]), d1 = lane_lo4(t[1][c]), d2 = lane_hi4(t[0][c]), d3 = lane_hi4(t[1][c]);
                    int y0, y1, y2, y3;
                    idct4(d0, d1, d2, d3, y0, y1, y2, y3);
                    rc[0][c] = ((cr ? y2 : y0) + 32) >> 6;
                    rc[1][c] = ((cr ? y3 : y1) + 32) >> 6;
                }
                // lossless: the raw levels, DC at (0,0) (transform.cc:453-455,860); an inter MB's
                // intra_chroma_pred_mode is DC (macroblock_t::init slice_data.cc:482), so
                // bypass_chroma (:802-822) copies
                if (byp) {
                    const int dcl = cb == 0 ? c00 : cb == 1 ? c01 : cb == 2 ? c10 : c11;
    #pragma unroll
                    for (int r = 0; r < 2; ++r)
    #pragma unroll
                        for (int c = 0; c < 2; ++c) rc[r][c] = (cr == 0 && cc == 0 && r == 0 && c == 0) ? dcl : raw[r][c];
                }
            }
            uint8_t* cdst = rmb + coff + pl * 64;
    #pragma unroll
            for (int r = 0; r < 2; ++r) {
                const uint32_t pr = predC[pl] >> (16 * r);
                const uint32_t wv = (uint32_t)clip255((int)(pr & 255) + rc[r][0]) |
                                    ((uint32_t)clip255((int)((pr >> 8) & 255) + rc[r][1]) << 8);
                *reinterpret_cast<uint16_t*>(cdst + r * 8) = (uint16_t)wv;
            }
        }
    }();
}

}  // namespace h264r
