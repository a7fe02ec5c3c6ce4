// mb_intra.h -- one intra macroblock per 64-lane wave (used by the level-scheduled
// k_intra_lvl and by the wavefront walk k_intra_pic).
//
//   Decoder::mb_pred_intra decoder.cc:170-208
//   IntraPrediction::intra_pred_{4x4,8x8,16x16,chroma} intra_prediction.cc:34-904
//   Transform::inverse_transform_{4x4,8x8,16x16,chroma} transform.cc:986-1049,
//   inverse_4x4 :597-641, inverse_8x8 :643-733, DC transforms :825-889.
//
// Structure (latency is what matters: the MBs of one dependency level run in
// parallel, each as a short chain of wave-synchronous steps):
//   1. every global load is issued up front: the MB record, the four neighbour
//      records (availability), the neighbour samples (row above x = -4..23,
//      column left, chroma likewise), the levels and scales;
//   2. the residual is computed in registers (lane = 4x4 block * 4 + row, four
//      samples per lane; rows in-lane, columns across the quad by DPP) -- the
//      8x8 transform goes through LDS;
//   3. I_16x16 and chroma predict in that same layout and store straight to the
//      picture; I_4x4 walks its 16 blocks as a wavefront over the block grid
//      (block (bx,by) at step bx + 2by: 10 steps, two blocks per step, one sample
//      per lane), I_8x8 its 4 blocks in order (one sample per lane);
//   4. every directional NxN mode is evaluated in one form: the neighbours along
//      the edge form a 1-D array e[] (left column bottom-up, corner, top row),
//      and each sample is a copy, a 2-tap or a [1,2,1] filter at an index of e[]
//      that depends on (mode, x, y) only (intra_nxn_tap below; spec 8.3.1.2.x /
//      8.3.2.2.x, intra_prediction.cc:189-346, 449-606).
#pragma once
#include "device_common.h"

namespace h264r {

constexpr int ITP = 32;   // luma tile pitch: x = -4..27 at byte x + 4, row y = -1..15 at (y + 1) * ITP
constexpr int ICP = 16;   // chroma tile pitch: x = -4..11

struct IntraScratch {
    alignas(16) uint8_t tile[17 * ITP];
    alignas(16) uint8_t ctile[2][9 * ICP];
    alignas(16) int res[16][16];          // luma residual (I_4x4 / I_8x8; every type when lossless)
    alignas(16) int cres[2][8][8];        // chroma residual of lossless MBs
    alignas(16) uint8_t fs[32];           // I_8x8 filtered neighbours: [3] Q, [4 + x] T[x], [20 + y] L[y]
    alignas(16) uint8_t fe[32];           // the same in e[] order: e[k] at [k + 1] (intra_nxn_tap)
};

DEV int ti(int x, int y) { return (y + 1) * ITP + x + 4; }          // luma tile index
DEV int ci(int x, int y) { return (y + 1) * ICP + x + 4; }          // chroma tile index

// (kind, index) of prediction sample (x, y) of an NxN block in directional mode
// `mode` (not DC): kind 0 = e[i], 1 = (e[i] + e[i+1] + 1) >> 1,
// 2 = (e[i-1] + 2 e[i] + e[i+1] + 2) >> 2.  e[] (3N + 3 entries): e[N - k] = L[k]
// (left column, k = 0..N-1), e[0] = L[N-1] again, e[N+1] = Q (corner),
// e[N+2+k] = T[k] (row above, k = 0..2N-1), e[3N+2] = T[2N-1] again -- the
// repeated ends give the (a + 3b + 2) >> 2 corner cases of modes 3 and 8.
template <int N>
constexpr __host__ __device__ void intra_nxn_tap(int mode, int x, int y, int& kind, int& i)
{
    switch (mode) {
    case 0: kind = 0; i = N + 2 + x; return;                                  // vertical
    case 1: kind = 0; i = N - y; return;                                      // horizontal
    case 3: kind = 2; i = N + 3 + x + y; return;                              // diagonal down left
    case 4: kind = 2; i = N + 1 + x - y; return;                              // diagonal down right
    case 5: {                                                                 // vertical right
        const int z = 2 * x - y;
        if (z >= 0) { kind = (z & 1) ? 2 : 1; i = N + 1 + x - (y >> 1); }
        else if (z == -1) { kind = 2; i = N + 1; }
        else { kind = 2; i = N + 2 + 2 * x - y; }
        return;
    }
    case 6: {                                                                 // horizontal down
        const int z = 2 * y - x;
        if (z >= 0) { if (z & 1) { kind = 2; i = N + 1 - y + (x >> 1); } else { kind = 1; i = N - y + (x >> 1); } }
        else if (z == -1) { kind = 2; i = N + 1; }
        else { kind = 2; i = N + x - 2 * y; }
        return;
    }
    case 7:                                                                   // vertical left
        if (y & 1) { kind = 2; i = N + 3 + x + (y >> 1); } else { kind = 1; i = N + 2 + x + (y >> 1); }
        return;
    default: {                                                                // horizontal up
        const int z = x + 2 * y;
        if (z < 2 * N - 3) { kind = (z & 1) ? 2 : 1; i = N - 1 - y - (x >> 1); }
        else if (z == 2 * N - 3) { kind = 2; i = 1; }
        else { kind = 0; i = 1; }
        return;
    }
    }
}

// The I_4x4 taps as tile offsets, one table per workgroup in LDS (copied from the
// compile-time INTRA_TAP_TABLE): entry mode * 32 + tv * 16 + (y * 4 + x) holds, for sample
// (x, y) of a 4x4 block in directional mode `mode`, the tile offsets (from the block
// origin, int8) of e[i - 1], e[i], e[i + 1] in bytes 0..2 and the kind in byte 3
// (intra_nxn_tap<4>); tv = 1 when the block's upper-right neighbours are available (the row
// above reaches x = 7, else it stops at 3).  e[k]: the left column bottom-up for k <= 5 (the
// corner at 5), then the row above.  DC entries are 0.  After them, the I_8x8 table: byte
// mode * 64 + (y * 8 + x) = i | kind << 5 of intra_nxn_tap<8> (I_8x8 reads e[] from S.fe, in
// order).  (Computed at run time in the kernels' prologue, the 8x8 part changed the walk's
// register allocation: 176 bytes of spills.)
constexpr int INTRA4_TAPS = 9 * 2 * 16;
constexpr int INTRA8_TAPS = 9 * 64 / 4;
constexpr int INTRA_NBR = INTRA4_TAPS + INTRA8_TAPS;   // + lane: the lane's neighbour-sample dword
constexpr int INTRA_TAPS = INTRA_NBR + 64;
struct IntraTapTable {
    uint32_t w[INTRA_TAPS];
};
constexpr IntraTapTable make_intra_taps()
{
    IntraTapTable t{};
    for (int e = 0; e < INTRA4_TAPS; ++e) {
        const int mode = e >> 5, tmax = (e & 16) ? 7 : 3, x = e & 3, y = (e >> 2) & 3;
        if (mode == 2) continue;
        int kind = 0, i = 0;
        intra_nxn_tap<4>(mode, x, y, kind, i);
        int o[3] = {0, 0, 0};
        for (int d = 0; d < 3; ++d) {
            const int k = d == 0 ? (i - 1 < 0 ? 0 : i - 1) : (d == 1 ? i : (i + 1 > 14 ? 14 : i + 1));
            const int up = k - 6 < tmax ? k - 6 : tmax;
            o[d] = k <= 5 ? (3 - (k - 1 > 0 ? k - 1 : 0)) * ITP - 1 : up - ITP;
        }
        t.w[e] = (uint32_t)(uint8_t)o[0] | ((uint32_t)(uint8_t)o[1] << 8) | ((uint32_t)(uint8_t)o[2] << 16) |
                 ((uint32_t)kind << 24);
    }
    for (int j = 0; j < 9 * 64; ++j) {
        const int mode = j >> 6;
        int kind = 0, i = 0;
        if (mode != 2) intra_nxn_tap<8>(mode, j & 7, (j >> 3) & 7, kind, i);
        t.w[INTRA4_TAPS + (j >> 2)] |= (uint32_t)(i | (kind << 5)) << (8 * (j & 3));
    }
    // the neighbour-sample dword of lane l (intra_head_samples): byte offset in the MB-tiled
    // neighbour MB (bits 0..8), its MB offset dx + 1 (bits 9..10) and dy + 1 (bit 11), the
    // lane loads (bit 12); bits 14..25: where the dword goes in IntraScratch -- the tile row
    // above (x = -4 .. 23 / chroma -4 .. 7) or, for the left columns, x = -4 .. -1 of the row
    // (the sample at -1; -4 .. -2 are not read); lanes without a sample write into S.res,
    // which every MB type rewrites before reading it
    for (int l = 0; l < 64; ++l) {
        int inner = 0, dx = 0, dy = 0, act = 0, at = 0;
        if (l < 7) {                                   // luma row above, x = -4 .. 23
            const int xr = 4 * l - 4;
            dx = xr < 0 ? -1 : (xr >> 4); dy = -1; inner = 15 * 16 + (xr & 15); act = 1;
            at = (int)offsetof(IntraScratch, tile) + 4 * l;
        } else if (l < 23) {                           // luma left column
            dx = -1; inner = (l - 7) * 16 + 12; act = 1;
            at = (int)offsetof(IntraScratch, tile) + (l - 7 + 1) * ITP;
        } else if (l < 29) {                           // chroma rows above, x = -4 .. 7
            const int k = l - 23, pl = k / 3, xc = 4 * (k % 3) - 4;
            dx = xc < 0 ? -1 : 0; dy = -1; inner = RECON_CB + pl * 64 + 7 * 8 + (xc & 7); act = 1;
            at = (int)offsetof(IntraScratch, ctile) + pl * 9 * ICP + 4 * (k % 3);
        } else if (l < 45) {                           // chroma left columns
            const int k = l - 29, pl = k >> 3;
            dx = -1; inner = RECON_CB + pl * 64 + (k & 7) * 8 + 4; act = 1;
            at = (int)offsetof(IntraScratch, ctile) + pl * 9 * ICP + ((k & 7) + 1) * ICP;
        } else {
            at = (int)offsetof(IntraScratch, res) + 4 * l;
        }
        t.w[INTRA_NBR + l] = (uint32_t)inner | ((uint32_t)(dx + 1) << 9) | ((uint32_t)(dy + 1) << 11) |
                             ((uint32_t)act << 12) | ((uint32_t)at << 14);
    }
    return t;
}
__device__ constexpr IntraTapTable INTRA_TAP_TABLE = make_intra_taps();
DEV const uint8_t* intra8_taps(const uint32_t* taps) { return reinterpret_cast<const uint8_t*>(taps + INTRA4_TAPS); }
DEV void intra4_tap_fill(uint32_t* tap4, int tid, int nthreads)
{
    for (int e = tid; e < INTRA_TAPS; e += nthreads) tap4[e] = INTRA_TAP_TABLE.w[e];
}

// kind 0 / 1 / 2 of intra_nxn_tap: all three forms, one kept by masks (a ternary chain on the
// lane's kind compiled to a tree of lane-divergent branches)
DEV int tap_apply(int kind, int a, int b, int c)
{
    const int t1 = (b + c + 1) >> 1, t2 = (a + 2 * b + c + 2) >> 2;
    const int m1 = -(kind & 1), m2 = -(kind >> 1);
    return ((b ^ ((b ^ t1) & m1)) & ~m2) | (t2 & m2);
}

DEV uint32_t lds_u32(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }
DEV int sum4(uint32_t w) { return (int)__builtin_amdgcn_sad_u8(w, 0u, 0u); }   // sum of the 4 bytes

// Every level and scale an intra MB's residual needs, loaded in ONE batch right after
// the MB record (the residual used to take two or three dependent round trips:
// luma levels, then the I_16x16 DC levels, then chroma -- profiles/r02_intra_phases.txt).
// Every load is unconditional: a lane without data reads the quant table and drops it
// (a load in a lane-divergent branch merges through a copy that waits for everything).
// (plain dwords: HIP's uint2 / uint4 unions in a struct passed around end up on the stack)
struct IntraLoads {
    uint32_t lev[2], sc[2]; // luma: 4x4 layout (lane = blk * 4 + row) or, I_8x8, (k, row, half)
    uint32_t dc[8];         // I_16x16: the 16 DC levels (raster)
    int dc_scale;           // I_16x16: scale4x4[0][0][qp % 6][0]
    uint32_t cdc[2];        // chroma: the plane's 4 DC levels
    int cdc_scale;
    uint32_t clev, csc;     // chroma AC: two levels and their scales
    bool lev_ok;            // lev holds coded levels (else: use 0)
};

// Branch-free: every address is a select, every load is issued, and a lane's "no data"
// case is applied where the value is used -- a load under a branch, or a select on a
// loaded value right after it, makes the compiler wait for it there.
// I4: the MB is known to be I_4x4 (intra_pair_i4): no I_8x8 layout, no I_16x16 DC loads.
template <bool I4 = false>
DEV IntraLoads intra_loads(const h264r_mb& m, const int16_t* __restrict__ lv, const h264r_quant* __restrict__ q, int lane)
{
    IntraLoads L;
    const int qp = m.qp_scaled[0], rem = qp % 6;
    const LevelOffs lo = level_offsets(m);
    const int16_t* dummy = &q->scale4x4[0][0][0][0];
    const bool i8 = !I4 && m.mb_type == H264R_I_8x8;
    // I_8x8 layout: k = lane >> 4, row, half; 4x4 layout: blk = lane >> 2, row
    const int k8 = lane >> 4, row8 = (lane >> 1) & 7, half8 = lane & 1;
    const int blk = lane >> 2, r4 = lane & 3, bx = blk & 3, by = blk >> 2;
    const int off = b8_offset(m.cbp, i8 ? k8 : (by >> 1) * 2 + (bx >> 1));
    const int within = i8 ? row8 * 8 + half8 * 4 : ((by & 1) * 2 + (bx & 1)) * 16 + r4 * 4;
    L.lev_ok = off >= 0;
    const uint2 lv2 = ld8(off >= 0 ? lv + off + within : dummy);
    const uint2 sc2 = ld8(i8 ? &q->scale8x8[0][0][rem][row8 * 8 + half8 * 4] : &q->scale4x4[0][0][rem][r4 * 4]);
    L.lev[0] = lv2.x; L.lev[1] = lv2.y; L.sc[0] = sc2.x; L.sc[1] = sc2.y;
    if (I4) {
        for (int k = 0; k < 8; ++k) L.dc[k] = 0u;
        L.dc_scale = 0;
    } else {
        const uint4* dcp = reinterpret_cast<const uint4*>(lo.ldc >= 0 ? lv + lo.ldc : dummy);
        const uint4 d0 = dcp[0], d1 = dcp[1];
        L.dc[0] = d0.x; L.dc[1] = d0.y; L.dc[2] = d0.z; L.dc[3] = d0.w;
        L.dc[4] = d1.x; L.dc[5] = d1.y; L.dc[6] = d1.z; L.dc[7] = d1.w;
        L.dc_scale = q->scale4x4[0][0][rem][0];
    }
    const int cpl = lane >> 5, cb = (lane >> 3) & 3, chalf = (lane >> 2) & 1, crow = lane & 3;
    const int qpc = (cpl ? m.qp_scaled[2] : m.qp_scaled[1]);
    const uint2 cd = ld8(lo.cdc >= 0 ? lv + lo.cdc + cpl * 4 : dummy);
    L.cdc[0] = cd.x; L.cdc[1] = cd.y;
    L.cdc_scale = q->scale4x4[0][1 + cpl][qpc % 6][0];
    L.clev = *reinterpret_cast<const uint32_t*>(lo.cac >= 0 ? lv + lo.cac + cpl * 64 + cb * 16 + crow * 4 + chalf * 2 : dummy);
    L.csc = *reinterpret_cast<const uint32_t*>(&q->scale4x4[0][1 + cpl][qpc % 6][crow * 4 + chalf * 2]);
    return L;
}

// Chroma residual of one MB (transform.cc:875-889 DC, inverse_4x4 for the AC blocks):
// lane = plane << 5 | blk << 3 | half << 2 | row, two samples (cols 2*half, +1).
DEV void chroma_res2(const h264r_mb& m, const IntraLoads& L, int lane, int (&resC)[2])
{
    const int cpl = lane >> 5, cb = (lane >> 3) & 3, chalf = (lane >> 2) & 1, crow = lane & 3;
    const int cbpc = m.cbp >> 4;
    resC[0] = resC[1] = 0;
    if (!cbpc) return;
    const int qpc = (cpl ? m.qp_scaled[2] : m.qp_scaled[1]), per = qpc / 6;
    int k0 = 0, k1 = 0;
    if (cbpc == 2) {
        k0 = dq4((int16_t)(L.clev & 0xFFFF), (int16_t)(L.csc & 0xFFFF), per);
        k1 = dq4((int16_t)(L.clev >> 16), (int16_t)(L.csc >> 16), per);
    }
    const int c00 = (int16_t)(L.cdc[0] & 0xFFFF), c01 = (int16_t)(L.cdc[0] >> 16);
    const int c10 = (int16_t)(L.cdc[1] & 0xFFFF), c11 = (int16_t)(L.cdc[1] >> 16);
    const int e00 = c00 + c01, e01 = c00 - c01, e10 = c10 + c11, e11 = c10 - c11;
    // f = (e00 or e01) +/- (e10 or e11) by cb's bits: arithmetic, not a branch tree
    const int ea = (cb & 1) ? e01 : e00, eb = (cb & 1) ? e11 : e10;
    const int f = ea + (eb ^ -(cb >> 1)) + (cb >> 1);
    const int kdc = ((f * L.cdc_scale) * (1 << per)) >> 5;
    k0 = (crow == 0 && chalf == 0) ? kdc : k0;
    const int d0 = lane_lo4(k0), d1 = lane_lo4(k1), d2 = lane_hi4(k0), d3 = lane_hi4(k1);   // chalf = lane bit 2
    int t[4];
    idct4(d0, d1, d2, d3, t[0], t[1], t[2], t[3]);
    const int u0 = chalf ? t[2] : t[0], u1 = chalf ? t[3] : t[1];
    resC[0] = idct4_col_row(quad_bcast<0>(u0), quad_bcast<1>(u0), quad_bcast<2>(u0), quad_bcast<3>(u0), crow);
    resC[1] = idct4_col_row(quad_bcast<0>(u1), quad_bcast<1>(u1), quad_bcast<2>(u1), quad_bcast<3>(u1), crow);
}

// Luma residual of an I_4x4 / I_16x16 MB in registers: lane = blk * 4 + row (blk
// raster over the 4x4 block grid), four samples.  I_16x16 DC: 4x4 Hadamard and
// scaling of transform_luma_dc (transform.cc:825-856), evaluated per lane.
template <bool I4 = false>
DEV void luma_res4_intra(const h264r_mb& m, const IntraLoads& L, int lane, int (&res)[4])
{
    const int blk = lane >> 2, r = lane & 3, bx = blk & 3, by = blk >> 2;
    const int qp = m.qp_scaled[0], per = qp / 6;
    const bool i16 = !I4 && m.mb_type == H264R_I_16x16;
    const uint32_t lev0 = L.lev_ok ? L.lev[0] : 0u, lev1 = L.lev_ok ? L.lev[1] : 0u;
    int d[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int l = (int16_t)((c & 2 ? lev1 : lev0) >> (16 * (c & 1)));
        const int s = (int16_t)((c & 2 ? L.sc[1] : L.sc[0]) >> (16 * (c & 1)));
        d[c] = dq4(l, s, per);
    }
    if (i16) {
        const uint32_t (&w)[8] = L.dc;
        const int mx = (0xA6C0 >> (4 * bx)) & 15, my = (0xA6C0 >> (4 * by)) & 15;   // Hadamard sign masks
        int f = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            int s = 0;
#pragma unroll
            for (int l = 0; l < 4; ++l) {
                const int v = (int16_t)(w[(4 * k + l) >> 1] >> (16 * (l & 1)));
                s += ((mx >> l) & 1) ? -v : v;
            }
            f += ((my >> k) & 1) ? -s : s;
        }
        const int scale = L.dc_scale;
        const int dc = qp >= 36 ? (f * scale) * (1 << (per - 6)) : (f * scale + (1 << (5 - per))) >> (6 - per);
        if (r == 0) d[0] = dc;
    }
    int t[4];
    idct4(d[0], d[1], d[2], d[3], t[0], t[1], t[2], t[3]);
#pragma unroll
    for (int c = 0; c < 4; ++c)
        res[c] = idct4_col_row(quad_bcast<0>(t[c]), quad_bcast<1>(t[c]), quad_bcast<2>(t[c]), quad_bcast<3>(t[c]), r);
}

// Luma residual of an I_8x8 MB (inverse_8x8, transform.cc:643-733) into S.res.
DEV void luma_res8_intra(const h264r_mb& m, const IntraLoads& L, int lane, IntraScratch& S)
{
    const int k = lane >> 4, row = (lane >> 1) & 7, half = lane & 1;
    const int qp = m.qp_scaled[0], per = qp / 6;
    const uint32_t lev0 = L.lev_ok ? L.lev[0] : 0u, lev1 = L.lev_ok ? L.lev[1] : 0u;
    int d[4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
        d[c] = dq8((int16_t)((c & 2 ? lev1 : lev0) >> (16 * (c & 1))),
                   (int16_t)((c & 2 ? L.sc[1] : L.sc[0]) >> (16 * (c & 1))), per);
    // row pass: the other half of my row is in lane ^ 1
    int in[8], out[8];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int o = __shfl_xor(d[c], 1);
        in[c] = half ? o : d[c];
        in[4 + c] = half ? d[c] : o;
    }
    idct8(in, out);
    int* dst = &S.res[(k >> 1) * 8 + row][(k & 1) * 8 + half * 4];
    *reinterpret_cast<int4*>(dst) = make_int4(out[half * 4], out[half * 4 + 1], out[half * 4 + 2], out[half * 4 + 3]);
    wave_sync();
    // column pass: lane = k * 16 + col * 2 + hv, outputs rows hv*4 .. hv*4 + 3
    {
        const int col = (lane >> 1) & 7, hv = lane & 1;
        const int x = (k & 1) * 8 + col, y0 = (k >> 1) * 8;
#pragma unroll
        for (int i = 0; i < 8; ++i) in[i] = S.res[y0 + i][x];
        idct8(in, out);
        wave_sync();                                   // every lane has read its column
#pragma unroll
        for (int i = 0; i < 4; ++i) S.res[y0 + hv * 4 + i][x] = (out[hv * 4 + i] + 32) >> 6;
    }
    wave_sync();
}

// Lossless DPCM of one line of n residual samples in place (transform.cc:736-822: a vertical
// mode accumulates down a column, a horizontal mode along a row; `step` is the distance of
// consecutive samples of the line).
DEV void dpcm_line(int* p, int step, int n)
{
    int acc = 0;
    for (int i = 0; i < n; ++i) { acc += p[i * step]; p[i * step] = acc; }
}

// Residual of a TransformBypassModeFlag MB (interpret_mb.cc:804): the levels are the
// residual (coeff_luma_ac / coeff_chroma_ac skip inverse_quantize, transform.cc:439-455; the
// DC transforms do nothing, :827,860), DPCM'd along the prediction direction of each block
// (bypass_4x4/8x8/16x16/chroma, :736-822, chosen by inverse_transform_* :986-1049).  The
// final luma residual is left in S.res (every MB type), I_16x16's also in resL (its
// register layout), chroma in resC.
DEV void intra_bypass_res(const h264r_mb& m, const int16_t* __restrict__ lv, int lane, IntraScratch& S, uint64_t ipw,
                          int (&resL)[4], int (&resC)[2])
{
    // the raw levels are loaded again here (rare MBs, L2-hot): keeping IntraLoads live into
    // this branch spilled the kernel
    const bool i8 = m.mb_type == H264R_I_8x8, i16 = m.mb_type == H264R_I_16x16;
    const LevelOffs lo = level_offsets(m);
    const int blk = lane >> 2, r = lane & 3, bx = blk & 3, by = blk >> 2;
    {
        const int k8 = lane >> 4, row8 = (lane >> 1) & 7, half8 = lane & 1;
        const int off = b8_offset(m.cbp, i8 ? k8 : (by >> 1) * 2 + (bx >> 1));
        const int within = i8 ? row8 * 8 + half8 * 4 : ((by & 1) * 2 + (bx & 1)) * 16 + r * 4;
        uint2 w = ld8(lv + (off >= 0 ? off + within : 0));
        if (off < 0) w = make_uint2(0, 0);
        int v[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = (int16_t)((c & 2 ? w.y : w.x) >> (16 * (c & 1)));
        if (i8) {
            *reinterpret_cast<int4*>(&S.res[(k8 >> 1) * 8 + row8][(k8 & 1) * 8 + half8 * 4]) = make_int4(v[0], v[1], v[2], v[3]);
        } else {
            if (i16 && r == 0) v[0] = lv[lo.ldc + 4 * by + bx];          // DC at (0,0)
            *reinterpret_cast<int4*>(&S.res[by * 4 + r][bx * 4]) = make_int4(v[0], v[1], v[2], v[3]);
        }
    }
    const int cpl = lane >> 5, cb = (lane >> 3) & 3, chalf = (lane >> 2) & 1, crow = lane & 3;
    const int cbpc = m.cbp >> 4;
    int c0 = 0, c1 = 0;
    if (cbpc == 2) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(lv + lo.cac + cpl * 64 + cb * 16 + crow * 4 + chalf * 2);
        c0 = (int16_t)(w & 0xFFFF);
        c1 = (int16_t)(w >> 16);
    }
    if (cbpc && crow == 0 && chalf == 0) c0 = lv[lo.cdc + cpl * 4 + cb];
    const int cy = (cb >> 1) * 4 + crow, cx = (cb & 1) * 4 + chalf * 2;
    S.cres[cpl][cy][cx] = c0;
    S.cres[cpl][cy][cx + 1] = c1;
    wave_sync();
    // one line per lane: vertical = 0 / horizontal = 1 for luma, 2 / 1 for chroma
    if (i8) {
        if (lane < 32) {
            const int b = lane >> 3, t = lane & 7, mode = (int)((ipw >> (4 * b)) & 15);
            int* o = &S.res[(b >> 1) * 8][(b & 1) * 8];
            if (mode == 0) dpcm_line(o + t, 16, 8);
            else if (mode == 1) dpcm_line(o + t * 16, 1, 8);
        }
    } else if (i16) {
        if (lane < 16) {
            if (m.i16_mode == 0) dpcm_line(&S.res[0][lane], 16, 16);
            else if (m.i16_mode == 1) dpcm_line(&S.res[lane][0], 1, 16);
        }
    } else {
        const int bk = (by >> 1) * 8 + (bx >> 1) * 4 + (by & 1) * 2 + (bx & 1);   // blkIdx
        const int mode = (int)((ipw >> (4 * bk)) & 15);
        int* o = &S.res[by * 4][bx * 4];
        if (mode == 0) dpcm_line(o + r, 16, 4);
        else if (mode == 1) dpcm_line(o + r * 16, 1, 4);
    }
    if (lane < 16) {
        int* o = &S.cres[lane >> 3][0][0];
        const int t = lane & 7;
        if (m.chroma_mode == 2) dpcm_line(o + t, 8, 8);
        else if (m.chroma_mode == 1) dpcm_line(o + t * 8, 1, 8);
    }
    wave_sync();
    if (i16) {
#pragma unroll
        for (int c = 0; c < 4; ++c) resL[c] = S.res[by * 4 + r][bx * 4 + c];
    }
    resC[0] = S.cres[cpl][cy][cx];
    resC[1] = S.cres[cpl][cy][cx + 1];
}

// The loads of one intra MB, in two stages: IntraHead needs nothing (neighbour samples,
// neighbour records, the MB record), IntraLoads needs the MB record (levels, scales).
// (Issuing both for the next MB while the current one is reconstructed held two MBs'
// records in SGPRs and spilled: 120 SGPRs, 55 VGPRs at 4 waves/SIMD.)
// The records are wave-uniform scalar loads (constant address space: immutable during
// a batch).
struct IntraHead {
    uint32_t nb;                 // this lane's neighbour sample dword (masked; INTRA_NBR)
    uint32_t nw0, nw2;           // lanes 0..3: neighbour record A, B, C, D (lane k): dwords 0 (type, flags) and 2 (cbp_blks, slice)
    bool nin;                    // lanes 0..3: that neighbour lies inside the picture
    h264r_mb m;
    int cip;
};

// The neighbour samples of MB (mbx, mby) for this lane: written by other waves (the row
// above) or by this one (the MB to the left), so loaded only once they are final.
DEV uint32_t intra_head_samples(const Geom& g, int pic, int mbx, int mby, int lane, uint8_t* recon, const uint32_t* taps)
{
    // ---- neighbour samples (in-picture addresses only; availability decides later which
    // of them are used): one dword load per lane (a left-column sample is the top byte of
    // the aligned dword that ends at x - 1; lanes with nothing to fetch read their own
    // MB's first row and drop it).  Each lane's neighbour MB and byte offset come from the
    // table (INTRA_NBR): a branch per lane group had cost the walk its exec-mask work.
    // (MB-tiled reconstruction, device_common.h: a dword never crosses an MB)
    const uint32_t e = taps[INTRA_NBR + lane];
    const int dx = (int)((e >> 9) & 3) - 1, dy = (int)((e >> 11) & 1) - 1;
    const int nx = mbx + dx;
    const bool want = ((e >> 12) & 1) && (dy == 0 || mby > 0) && nx >= 0 && nx < g.wmb;
    const int a = want ? (mby + dy) * g.wmb + nx : mby * g.wmb + mbx;
    const uint8_t* src = recon_mb(recon, g, pic, a) + (want ? (int)(e & 511) : 0);
    return *as_global(src) & (0u - (uint32_t)want);    // arithmetic, not a select: no branch
}

// The records of MB (mbx, mby) and its neighbours: immutable during a batch, so the walk
// loads them (and the levels they point to) before it waits for the row above.  The
// neighbour records A, B, C, D go to lanes 0..3 by one vector load each (as scalar loads
// they took SGPRs the walk does not have: the compiler issued them one at a time, each
// behind its own wait).
DEV void intra_head_records(const h264r_batch& b, const Geom& g, int pic, int mbx, int mby, int lane, IntraHead& h)
{
    const int a = mby * g.wmb + mbx;
    const h264r_mb* mbs = b.mbs + (size_t)pic * g.nmb;
    // neighbour records (get_neighbour + slice check + constrained intra,
    // intra_prediction.cc:142-168 / 629-651 / 753-777) and the MB record
    const int k = lane & 3;
    const int nx = mbx + (k == 0 || k == 3 ? -1 : (k == 2 ? 1 : 0)), ny = mby - (k == 0 ? 0 : 1);
    h.nin = nx >= 0 && ny >= 0 && nx < g.wmb && ny < g.hmb;
    const uint2 w = *reinterpret_cast<const uint2*>(&mbs[h.nin ? ny * g.wmb + nx : a]);   // dwords 0, 1
    h.nw0 = w.x;
    h.nw2 = reinterpret_cast<const uint32_t*>(&mbs[h.nin ? ny * g.wmb + nx : a])[2];
    h.cip = ld_const(&b.pics[pic].constrained_intra_pred);
    h.m = load_mb_const(&mbs[a]);
}

DEV IntraHead intra_head(const h264r_batch& b, const Geom& g, int pic, int mbx, int mby, int lane, uint8_t* recon,
                         const uint32_t* taps)
{
    IntraHead h;
    h.nb = intra_head_samples(g, pic, mbx, mby, lane, recon, taps);
    intra_head_records(b, g, pic, mbx, mby, lane, h);
    return h;
}

DEV IntraLoads intra_body_loads(const h264r_batch& b, int pic, const IntraHead& h, int lane)
{
    return intra_loads(h.m, b.levels + h.m.coef_off, &b.quant[pic], lane);
}

// What the I_4x4 steps need of an MB: its neighbours' availability and its 16 modes.
struct I4Mb {
    int avA, avB, avC;
    uint64_t ipw;
};

// The I_4x4 steps of two MBs at once: MB A on lanes 0..31 (tiles SA), MB B on lanes 32..63
// (SB), in the slot layout of intra_mb_compute's I_4x4 steps.  The two MBs' modes and availability differ, so a lane
// derives its block's from its own MB's (per-lane) mode word and availability bits and the
// step's compile-time block coordinates; whether the step needs the DC sums or the directional
// taps is one ballot each.
DEV void intra4_steps_pair(int lane, IntraScratch& SA, IntraScratch& SB, const I4Mb& A, const I4Mb& B, const uint32_t* tap4)
{
    const int slot = (lane >> 4) & 1, x = lane & 3, y = (lane >> 2) & 3;
    const bool mbB = lane >= 32;
    IntraScratch& S = mbB ? SB : SA;
    const int soff = y * ITP + x, roff = y * 16 + x, pos = lane & 15;
    const uint64_t ipw = mbB ? B.ipw : A.ipw;
    const int avA = mbB ? B.avA : A.avA, avB = mbB ? B.avB : A.avB, avC = mbB ? B.avC : A.avC;
    // this lane's block of step s: slot 0 = (s & 1) + 2, (s >> 1) - 1; slot 1 = s & 1, s >> 1
    struct Lb { bool on; int mode, aA, aB, tv, pb, rb; };
    auto lane_blk = [&](int s) -> Lb {
        const int by0 = (s >> 1) - 1, bx0 = (s & 1) + 2, by1 = s >> 1, bx1 = s & 1;
        const bool ok0 = by0 >= 0, ok1 = by1 <= 3;
        auto bk_of = [](int bx, int by) { return (by >> 1) * 8 + (bx >> 1) * 4 + (by & 1) * 2 + (bx & 1); };   // blkIdx
        auto tvc = [](int bx, int by) { return (bx * 4 + 4 < 16) && !(bx == 1 && (by == 1 || by == 3)); };  // :154
        Lb l;
        l.on = slot ? ok1 : ok0;
        const int bk = slot ? (ok1 ? bk_of(bx1, by1) : 0) : (ok0 ? bk_of(bx0, by0) : 0);
        l.mode = l.on ? (int)((ipw >> (4 * bk)) & 15) : 0;
        const int bx = slot ? bx1 : bx0, by = slot ? by1 : by0;
        l.aA = bx > 0 ? 1 : avA;
        l.aB = by > 0 ? 1 : avB;
        // tv: the block's upper-right neighbours available (row 0: from B / C; below: fixed)
        const int tv0 = by0 == 0 ? (bx0 < 3 ? avB : avC) : (int)tvc(bx0, by0);
        const int tv1 = by1 == 0 ? (bx1 < 3 ? avB : avC) : (int)tvc(bx1, by1);
        l.tv = l.on ? (slot ? tv1 : tv0) : 0;
        l.pb = slot ? (ok1 ? ti(bx1 * 4, by1 * 4) : ti(4, 4)) : (ok0 ? ti(bx0 * 4, by0 * 4) : ti(4, 4));
        l.rb = slot ? (ok1 ? by1 * 64 + bx1 * 4 : 0) : (ok0 ? by0 * 64 + bx0 * 4 : 0);
        return l;
    };
    Lb cur = lane_blk(0);
    uint32_t ent_next = tap4[cur.mode * 32 + cur.tv * 16 + pos];
    int res_next = (&S.res[0][0])[cur.rb + roff];
#pragma unroll
    for (int s = 0; s < 10; ++s) {
        const Lb l = cur;
        const uint32_t ent = ent_next;
        const int rv = res_next;
        int tp = 0, dc = 0;
        if (__ballot(l.on && l.mode != 2) != 0) {
            const int e0 = S.tile[l.pb + (int)(int8_t)ent], e1 = S.tile[l.pb + (int)(int8_t)(ent >> 8)];
            const int e2 = S.tile[l.pb + (int)(int8_t)(ent >> 16)];
            tp = tap_apply((int)(ent >> 24), e0, e1, e2);
        }
        if (__ballot(l.on && l.mode == 2) != 0) {                 // DC (:214-229)
            const int st = sum4(lds_u32(&S.tile[l.pb - ITP]));
            const int sl = S.tile[l.pb - 1] + S.tile[l.pb + ITP - 1] + S.tile[l.pb + 2 * ITP - 1] + S.tile[l.pb + 3 * ITP - 1];
            const int mA = -l.aA, mB = -l.aB, dsh = 1 + l.aA + l.aB;
            dc = (((sl & mA) + (st & mB) + (1 << (dsh - 1))) >> dsh) + (128 & ~(mA | mB));
        }
        const int p = l.mode == 2 ? dc : tp;
        const int v = clip255(p + rv);                            // residual: 0 in uncoded blocks
        if (l.on) S.tile[l.pb + soff] = (uint8_t)v;
        if (s < 9) {
            cur = lane_blk(s + 1);
            ent_next = tap4[cur.mode * 32 + cur.tv * 16 + pos];
            res_next = (&S.res[0][0])[cur.rb + roff];
        }
        wave_sync();
    }
}

// IntraPrediction::Chroma (intra_prediction.cc:748-894) + construction_chroma of one MB, in the
// chroma residual layout (lane = plane << 5 | blk << 3 | half << 2 | row, two samples).
DEV void intra_chroma(const h264r_mb& m, int avA, int avB, int lane, const IntraScratch& S, const int (&resC)[2], uint8_t* rmb)
{
    const int pl = lane >> 5, cb = (lane >> 3) & 3, chalf = (lane >> 2) & 1, crow = lane & 3;
    const int y = (cb >> 1) * 4 + crow, x0 = (cb & 1) * 4 + chalf * 2;
    const uint8_t* C = S.ctile[pl];
    const int mode = m.chroma_mode;
    int p[2];
    if (mode == 0) {
        // per 4x4 block: both sums read, the available ones selected (no lane-divergent branch)
        const int xO = x0 & 4, yO = y & 4;
        const bool diag = (xO == 0) == (yO == 0);                  // blocks (0,0) and (4,4)
        const int aA = diag || xO == 0 ? avA : (avB ? 0 : avA);
        const int aB = diag || xO > 0 ? avB : (avA ? 0 : avB);
        const int sl = C[ci(-1, yO)] + C[ci(-1, yO + 1)] + C[ci(-1, yO + 2)] + C[ci(-1, yO + 3)];
        const int st = sum4(lds_u32(&C[ci(xO, -1)]));
        const int sum = (aA ? sl : 0) + (aB ? st : 0) + (aA ? 2 : 0) + (aB ? 2 : 0);
        const int v = aA || aB ? sum >> (1 + aA + aB) : 128;
        p[0] = p[1] = v;
    } else if (mode == 1) {
        p[0] = p[1] = C[ci(-1, y)];
    } else if (mode == 2) {
        p[0] = C[ci(x0, -1)];
        p[1] = C[ci(x0 + 1, -1)];
    } else {
        int Hs = 0, Vs = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            Hs += (k + 1) * (C[ci(4 + k, -1)] - C[ci(2 - k, -1)]);
            Vs += (k + 1) * (C[ci(-1, 4 + k)] - C[ci(-1, 2 - k)]);
        }
        const int pa = 16 * (C[ci(-1, 7)] + C[ci(7, -1)]);
        const int pb = (34 * Hs + 32) >> 6, pc = (34 * Vs + 32) >> 6;
#pragma unroll
        for (int c = 0; c < 2; ++c) p[c] = clip255((pa + pb * (x0 + c - 3) + pc * (y - 3) + 16) >> 5);
    }
    const uint32_t w = (uint32_t)clip255(p[0] + resC[0]) | ((uint32_t)clip255(p[1] + resC[1]) << 8);
    *reinterpret_cast<uint16_t*>(rmb + RECON_CB + pl * 64 + y * 8 + x0) = (uint16_t)w;
}

// Intra MB (mbx, mby) of picture `pic` from its loads (no-op for inter / I_PCM MBs); one
// wave.  tph (trace builds): s_memtime at the phase boundaries [record known, residual,
// tiles, prediction, end].
DEV void intra_mb_compute(const h264r_batch& b, const Geom& g, int pic, int mbx, int mby, int lane, IntraScratch& S,
                          const uint32_t* tap4, const IntraHead& hd, const IntraLoads& ld, uint8_t* recon,
                          unsigned long long* tph = nullptr)
{
#define INTRA_STAMP(k) do { if (tph) tph[k] = __builtin_amdgcn_s_memtime(); } while (0)
    uint8_t* const rmb = recon_mb(recon, g, pic, mby * g.wmb + mbx);      // MB-tiled (device_common.h)
    const h264r_mb& m = hd.m;
    const uint32_t nb = hd.nb;
    // the 16 intra 4x4 / 4 intra 8x8 modes as one 64-bit word (h264r_mb::ipred, dwords 5-6):
    // indexed per lane by shifts, not through the record's bytes (that puts it on the stack)
    const uint64_t ipw = (uint64_t)reinterpret_cast<const uint32_t*>(&m)[5] |
                         ((uint64_t)reinterpret_cast<const uint32_t*>(&m)[6] << 32);
    if (!mb_is_intra(m) || m.mb_type == H264R_I_PCM) return;
    INTRA_STAMP(0);
    // availability of neighbour k from lane k's record, all four in one mask (wave-uniform)
    const bool av = lane < 4 && hd.nin && (int)(hd.nw2 >> 16) == (int)m.slice &&
                    !(hd.cip && !((hd.nw0 >> 8) & H264R_MBF_INTRA));
    const uint32_t avm = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)__ballot(av));
    const int avA = avm & 1, avB = (avm >> 1) & 1, avC = (avm >> 2) & 1, avD = (avm >> 3) & 1;
    const bool i16 = m.mb_type == H264R_I_16x16, i8 = m.mb_type == H264R_I_8x8;

    // ---- residual (registers; 8x8 via LDS; lossless MBs via LDS)
    const bool byp = (m.flags & H264R_MBF_BYPASS) != 0;
    int resL[4] = {0, 0, 0, 0}, resC[2] = {0, 0};
    if (!i8) luma_res4_intra(m, ld, lane, resL);
    chroma_res2(m, ld, lane, resC);
    if (tph) { asm volatile("; stamp after residual" ::"v"(resL[0]), "v"(resC[0])); }
    INTRA_STAMP(1);

    // ---- neighbours into the tiles
    // (one dword store per lane at its INTRA_NBR offset: no lane-group branches)
    *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(&S) + ((tap4[INTRA_NBR + lane] >> 14) & 4095)) = nb;
    if (byp) intra_bypass_res(m, b.levels + m.coef_off, lane, S, ipw, resL, resC);   // S.res too
    else if (i8) luma_res8_intra(m, ld, lane, S);      // includes wave_syncs
    else if (!i16) {
        const int blk = lane >> 2, r = lane & 3;
        *reinterpret_cast<int4*>(&S.res[(blk >> 2) * 4 + r][(blk & 3) * 4]) = make_int4(resL[0], resL[1], resL[2], resL[3]);
    }
    wave_sync();
    INTRA_STAMP(2);
    const int cbpl = m.cbp & 15;

    if (i16) {
        // Intra16x16 (intra_prediction.cc:668-735) + construction_16x16 (transform.cc:940-959),
        // in the residual layout: row y = by * 4 + r, cols x0 .. x0 + 3.
        const int blk = lane >> 2, r = lane & 3, y = (blk >> 2) * 4 + r, x0 = (blk & 3) * 4;
        const int mode = m.i16_mode;
        int p[4];
        if (mode == 0) {
            const uint32_t w = lds_u32(&S.tile[ti(x0, -1)]);
#pragma unroll
            for (int c = 0; c < 4; ++c) p[c] = (w >> (8 * c)) & 255;
        } else if (mode == 1) {
            p[0] = p[1] = p[2] = p[3] = S.tile[ti(-1, y)];
        } else if (mode == 2) {
            int sum = 0, dc = 128;
            if (avB)
#pragma unroll
                for (int k = 0; k < 4; ++k) sum += sum4(lds_u32(&S.tile[ti(4 * k, -1)]));
            if (avA)
#pragma unroll
                for (int k = 0; k < 16; ++k) sum += S.tile[ti(-1, k)];
            if (avA || avB) dc = (sum + (avA ? 8 : 0) + (avB ? 8 : 0)) >> (3 + avA + avB);
            p[0] = p[1] = p[2] = p[3] = dc;
        } else {
            int Hs = 0, Vs = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                Hs += (k + 1) * (S.tile[ti(8 + k, -1)] - S.tile[ti(6 - k, -1)]);
                Vs += (k + 1) * (S.tile[ti(-1, 8 + k)] - S.tile[ti(-1, 6 - k)]);
            }
            const int pa = 16 * (S.tile[ti(-1, 15)] + S.tile[ti(15, -1)]);
            const int pb = (5 * Hs + 32) >> 6, pc = (5 * Vs + 32) >> 6;
#pragma unroll
            for (int c = 0; c < 4; ++c) p[c] = clip255((pa + pb * (x0 + c - 7) + pc * (y - 7) + 16) >> 5);
        }
        uint32_t w = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) w |= (uint32_t)clip255(p[c] + resL[c]) << (8 * c);
        *reinterpret_cast<uint32_t*>(rmb + y * 16 + x0) = w;
    } else if (i8) {
        // I_8x8, its 4 blocks in order (unrolled: each block's availability and mode are
        // wave-uniform).  The reference sample filter (intra_prediction.cc:413-447) runs on
        // lanes 0..24 over the sequence s = L[7..0], Q, T[0..15] (s[j] = e[j + 1]): every
        // filtered sample is (A + 2 B + C + 2) >> 2 of its two sequence neighbours, a
        // neighbour outside the sequence or unavailable being B itself -- one form, selects
        // instead of lane-divergent branches.  The result goes to S.fe in e[] order (e[k] at
        // fe[k + 1], the repeated ends included; the taps read fe[i .. i + 2]) and to S.fs
        // (the DC sums).
        const uint8_t* t8 = intra8_taps(tap4) + lane;                // + mode * 64: my sample's entry
        const int j = min(lane, 24);
        const int at_e = lane < 25 ? j + 2 : 31, at_dup = lane == 0 ? 1 : (lane == 24 ? 27 : 31);
        const int at_fs = lane >= 25 ? 31 : (j < 8 ? 27 - j : (j == 8 ? 3 : j - 5));
#pragma unroll
        for (int blk = 0; blk < 4; ++blk) {
            const int xO = (blk & 1) * 8, yO = (blk >> 1) * 8;
            const int aA = xO > 0 ? 1 : avA, aB = yO > 0 ? 1 : avB;
            const int aD = (xO > 0 && yO > 0) ? 1 : (xO == 0 && yO == 0) ? avD : (xO == 0 ? avA : avB);
            const int aC = yO > 0 ? (xO == 0) : (xO == 0 ? avB : avC);   // intra_prediction.cc:370-376
            const int mode = (int)((ipw >> (4 * blk)) & 15);
            const int tcap = aC ? 15 : 7;                                // p(x,-1) substitution :404-407
            const int bo = ti(xO, yO);
            auto off = [&](int k) -> int {                               // tile offset of s[k] from the block origin
                int l = (7 - k) * ITP - 1, t = min(k - 9, tcap) - ITP;
                asm volatile("" : "+v"(l), "+v"(t));
                return k < 8 ? l : t;
            };
            const int B = S.tile[bo + off(j)];
            int A = S.tile[bo + off(max(j - 1, 0))], C = S.tile[bo + off(min(j + 1, 24))];
            A = (j == 9 && !aD) || (j == 8 && !aA) ? B : A;
            C = (j == 7 && !aD) || (j == 8 && !aB) ? B : C;
            const bool valid = j < 8 ? aA : (j == 8 ? aD : aB);
            const int v = valid ? (A + 2 * B + C + 2) >> 2 : 0;
            S.fe[at_e] = (uint8_t)v;
            S.fe[at_dup] = (uint8_t)v;
            S.fs[at_fs] = (uint8_t)v;
            wave_sync();
            {
                const int x = lane & 7, y = lane >> 3;
                int p;
                if (mode == 2) {                                       // DC (intra_prediction.cc:480-497)
                    const int st = sum4(lds_u32(&S.fs[4])) + sum4(lds_u32(&S.fs[8]));
                    const int sl = sum4(lds_u32(&S.fs[20])) + sum4(lds_u32(&S.fs[24]));
                    p = aA && aB ? (st + sl + 8) >> 4 : aB ? (st + 4) >> 3 : aA ? (sl + 4) >> 3 : 128;
                } else {
                    const int ent = t8[mode * 64], kind = ent >> 5, i = ent & 31;
                    const uint8_t* e = &S.fe[i];                       // e[i - 1], e[i], e[i + 1]
                    p = tap_apply(kind, e[0], e[1], e[2]);
                }
                const int v = (cbpl >> blk) & 1 ? clip255(p + S.res[yO + y][xO + x]) : p;
                S.tile[ti(xO + x, yO + y)] = (uint8_t)v;
            }
            wave_sync();
        }
    } else {
        // I_4x4: block (bx, by) at step bx + 2 by, two blocks per step: lanes 0..15 (slot 0) the
        // one with the larger bx, lanes 16..31 (slot 1) the other.  The steps are unrolled, so
        // each slot's block, availability and mode are wave-uniform (scalar) and a lane only
        // selects between the two slots' values; every per-lane expression is a select, not a
        // branch (a lane-divergent branch runs both sides anyway, plus the exec-mask work).
        // A sample's three e[] taps come as tile offsets from the workgroup's table (tap4:
        // intra4_tap_fill), the DC sums and the directional taps each run only when a slot of
        // the step needs them (scalar branches on the two modes).
        const int slot = (lane >> 4) & 1, x = lane & 3, y = (lane >> 2) & 3;
        const bool half = lane < 32;
        const int soff = y * ITP + x, roff = y * 16 + x, pos = lane & 15;
        // the two slots of step s: block coordinates (compile time), mode, availability (scalar);
        // an absent slot has mode 0 (no DC work) and reads around an interior origin
        struct StepPar { bool ok0, ok1; int m0, a0, b0, t0, m1, a1, b1, t1, base0, base1, rb0, rb1; };
        auto step_par = [&](int s) -> StepPar {
            StepPar q;
            const int by0 = (s >> 1) - 1, bx0 = (s & 1) + 2, by1 = s >> 1, bx1 = s & 1;
            q.ok0 = by0 >= 0; q.ok1 = by1 <= 3;
            auto blk_par = [&](int bx, int by, int& mode, int& aA, int& aB, int& tv) {
                const int xO = bx * 4, yO = by * 4;
                const int bk = (by >> 1) * 8 + (bx >> 1) * 4 + (by & 1) * 2 + (bx & 1);   // blkIdx
                aA = xO > 0 ? 1 : avA;
                aB = yO > 0 ? 1 : avB;
                tv = yO == 0 ? (xO + 4 < 16 ? avB : avC) : ((xO + 4 < 16) && !(xO == 4 && (yO == 4 || yO == 12)));   // :154
                mode = (int)((ipw >> (4 * bk)) & 15);
            };
            q.m0 = q.a0 = q.b0 = q.t0 = q.m1 = q.a1 = q.b1 = q.t1 = 0;
            if (q.ok0) blk_par(bx0, by0, q.m0, q.a0, q.b0, q.t0);
            if (q.ok1) blk_par(bx1, by1, q.m1, q.a1, q.b1, q.t1);
            q.base0 = q.ok0 ? ti(bx0 * 4, by0 * 4) : ti(4, 4);
            q.base1 = q.ok1 ? ti(bx1 * 4, by1 * 4) : ti(4, 4);
            q.rb0 = q.ok0 ? by0 * 64 + bx0 * 4 : 0;
            q.rb1 = q.ok1 ? by1 * 64 + bx1 * 4 : 0;
            return q;
        };
        // what a step reads that no step writes -- its table entry and residual sample -- is
        // read during the step before, so a step waits on one LDS round trip (the tile reads)
        auto step_ent = [&](const StepPar& q) -> uint32_t { return tap4[(slot ? q.m1 * 32 + q.t1 * 16 : q.m0 * 32 + q.t0 * 16) + pos]; };
        auto step_res = [&](const StepPar& q) -> int { return (&S.res[0][0])[(slot ? q.rb1 : q.rb0) + roff]; };
        uint32_t ent_next = step_ent(step_par(0));
        int res_next = step_res(step_par(0));
#pragma unroll
        for (int s = 0; s < 10; ++s) {
            const StepPar q = step_par(s);
            const uint32_t ent = ent_next;
            const int rv = res_next;
            const bool on = half && (slot ? q.ok1 : q.ok0);
            const int mode = slot ? q.m1 : q.m0, pb = slot ? q.base1 : q.base0;
            int tp = 0, dc = 0;
            if (q.m0 != 2 || q.m1 != 2) {
                const int e0 = S.tile[pb + (int)(int8_t)ent], e1 = S.tile[pb + (int)(int8_t)(ent >> 8)];
                const int e2 = S.tile[pb + (int)(int8_t)(ent >> 16)];
                tp = tap_apply((int)(ent >> 24), e0, e1, e2);
            }
            if (q.m0 == 2 || q.m1 == 2) {                            // DC (intra_prediction.cc:214-229)
                const int aA = slot ? q.a1 : q.a0, aB = slot ? q.b1 : q.b0;
                const int st = sum4(lds_u32(&S.tile[pb - ITP]));
                const int sl = S.tile[pb - 1] + S.tile[pb + ITP - 1] + S.tile[pb + 2 * ITP - 1] + S.tile[pb + 3 * ITP - 1];
                // by masks: the available sums, shifted by 2 or 3, 128 when neither side is
                const int mA = -aA, mB = -aB, dsh = 1 + aA + aB;
                dc = (((sl & mA) + (st & mB) + (1 << (dsh - 1))) >> dsh) + (128 & ~(mA | mB));
            }
            const int p = mode == 2 ? dc : tp;
            const int v = clip255(p + rv);                           // residual: 0 in uncoded blocks
            if (on) S.tile[pb + soff] = (uint8_t)v;
            if (s < 9) {
                const StepPar qn = step_par(s + 1);
                ent_next = step_ent(qn);
                res_next = step_res(qn);
            }
            wave_sync();
        }
    }
    INTRA_STAMP(3);
    if (!i16) {
        const int y = lane >> 2, x0 = (lane & 3) * 4;
        *reinterpret_cast<uint32_t*>(rmb + y * 16 + x0) = lds_u32(&S.tile[ti(x0, y)]);
    }

    // ---- chroma: IntraPrediction::Chroma (intra_prediction.cc:748-894) + construction_chroma
    intra_chroma(m, avA, avB, lane, S, resC, rmb);
    INTRA_STAMP(4);
#undef INTRA_STAMP
}

// The class of MB the level lists pair (k_level): I_4x4, not lossless.
DEV bool intra_pairable(const h264r_mb& m)
{
    return mb_is_intra(m) && m.mb_type == H264R_I_4x4 && !(m.flags & H264R_MBF_BYPASS);
}

// Two I_4x4 MBs (intra_pairable) of one dependency level in one wave -- independent, since an
// intra neighbour would put one a level below the other.  The loads of both come first; the
// residual, the neighbour tiles, the luma stores and the chroma run per MB in the single-MB
// layouts, and the ten I_4x4 steps -- four fifths of an I_4x4 MB's time in one wave
// (profiles/r05_ad_intra_trace.txt), with half the wave idle -- once for both: MB A on lanes
// 0..31, MB B on lanes 32..63 (intra4_steps_pair).  k = pic * nmb + MB address.  Returns
// false, having stored nothing, when either MB is not pairable.
DEV bool intra_pair_i4(const h264r_batch& b, const Geom& g, uint32_t kA, uint32_t kB, int lane, IntraScratch& SA,
                       IntraScratch& SB, const uint32_t* tap4, uint8_t* recon)
{
    const int picA = (int)(kA / (unsigned)g.nmb), aA = (int)(kA % (unsigned)g.nmb);
    const int picB = (int)(kB / (unsigned)g.nmb), aB = (int)(kB % (unsigned)g.nmb);
    const int xA = aA % g.wmb, yA = aA / g.wmb, xB = aB % g.wmb, yB = aB / g.wmb;
    const IntraHead hA = intra_head(b, g, picA, xA, yA, lane, recon, tap4);
    const IntraHead hB = intra_head(b, g, picB, xB, yB, lane, recon, tap4);
    if (!intra_pairable(hA.m) || !intra_pairable(hB.m)) return false;
    const IntraLoads lA = intra_loads<true>(hA.m, b.levels + hA.m.coef_off, &b.quant[picA], lane);
    const IntraLoads lB = intra_loads<true>(hB.m, b.levels + hB.m.coef_off, &b.quant[picB], lane);
    // per MB: availability (one ballot), residual (luma into S.res, chroma in registers),
    // neighbour samples into the tile
    auto pre = [&](const IntraHead& hd, const IntraLoads& ld, IntraScratch& S, int (&resC)[2]) -> I4Mb {
        const h264r_mb& m = hd.m;
        const bool av = lane < 4 && hd.nin && (int)(hd.nw2 >> 16) == (int)m.slice &&
                        !(hd.cip && !((hd.nw0 >> 8) & H264R_MBF_INTRA));
        const uint32_t avm = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)__ballot(av));
        int resL[4];
        luma_res4_intra<true>(m, ld, lane, resL);
        chroma_res2(m, ld, lane, resC);
        *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(&S) + ((tap4[INTRA_NBR + lane] >> 14) & 4095)) = hd.nb;
        const int blk = lane >> 2, r = lane & 3;
        *reinterpret_cast<int4*>(&S.res[(blk >> 2) * 4 + r][(blk & 3) * 4]) = make_int4(resL[0], resL[1], resL[2], resL[3]);
        const uint64_t ipw = (uint64_t)reinterpret_cast<const uint32_t*>(&m)[5] |
                             ((uint64_t)reinterpret_cast<const uint32_t*>(&m)[6] << 32);
        return I4Mb{(int)(avm & 1), (int)((avm >> 1) & 1), (int)((avm >> 2) & 1), ipw};
    };
    int resCA[2], resCB[2];
    const I4Mb pA = pre(hA, lA, SA, resCA);
    const I4Mb pB = pre(hB, lB, SB, resCB);
    wave_sync();
    intra4_steps_pair(lane, SA, SB, pA, pB, tap4);
    uint8_t* const rA = recon_mb(recon, g, picA, aA);
    uint8_t* const rB = recon_mb(recon, g, picB, aB);
    {
        const int y = lane >> 2, x0 = (lane & 3) * 4;
        *reinterpret_cast<uint32_t*>(rA + y * 16 + x0) = lds_u32(&SA.tile[ti(x0, y)]);
        *reinterpret_cast<uint32_t*>(rB + y * 16 + x0) = lds_u32(&SB.tile[ti(x0, y)]);
    }
    intra_chroma(hA.m, pA.avA, pA.avB, lane, SA, resCA, rA);
    intra_chroma(hB.m, pB.avA, pB.avB, lane, SB, resCB, rB);
    return true;
}

// Loads then reconstruction of one intra MB (the walk, k_intra_pic).
DEV void intra_mb2(const h264r_batch& b, const Geom& g, int pic, int mbx, int mby, int lane, IntraScratch& S,
                   const uint32_t* tap4, uint8_t* recon, unsigned long long* tph = nullptr)
{
    const IntraHead hd = intra_head(b, g, pic, mbx, mby, lane, recon, tap4);
    if (!mb_is_intra(hd.m) || hd.m.mb_type == H264R_I_PCM) return;
    const IntraLoads ld = intra_body_loads(b, pic, hd, lane);
    intra_mb_compute(b, g, pic, mbx, mby, lane, S, tap4, hd, ld, recon, tph);
}

}  // namespace h264r
