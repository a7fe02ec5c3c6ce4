// k_chroma422.hip -- the chroma planes of 4:2:2 pictures (chroma_format_idc 2), gfx950.
//
// A 4:2:2 MB has 8 x 16 chroma samples per plane (MbHeightC 16): eight 4x4 blocks, a 2x4 DC
// matrix, vertical chroma vectors in quarter rows.  Its luma is the 4:2:0 luma, so a 4:2:2 batch
// runs (h264r_host.hip run_422):
//   1. the 4:2:0 launch sequence on the luma plane (k_derive444 plane 0: chroma stripped from the
//      records, the chroma of that pass goes to scratch) -- it also leaves the deblocking records
//      (DbInfo, mb_deblock.h) of every MB;
//   2. k_c422_inter, k_c422_intra: the reconstruction of both chroma planes, raster into the output
//      planes -- every inter and I_PCM MB at once, then the intra MBs in a row walk;
//   3. k_c422_db: their deblocking, in place, from those records.
// The reference paths (R/src/codec/h264/decoder/, H/ below):
//   prediction   IntraPrediction::Chroma intra_prediction.cc:748-894 (the plane constants
//                xCF 0 / yCF 4, :871-894); get_block_chroma inter_prediction.cc:342-406 (yAL =
//                mv >> 2, yFracC = (mv & 3) << 1, :381-383) with mc_prediction / bi_prediction :53-156
//   residual     coeff_chroma_ac / inverse_quantize transform.cc:394-456, transform_chroma_dc
//                :858-910 (ihadamard_2x4 :483-513; qP = qp_scaled[pl], see below), inverse_4x4 per
//                block and bypass_chroma for lossless MBs (inverse_transform_chroma :1033-1049),
//                construction_chroma; I_PCM mb_pred_ipcm decoder.cc:149-168
//   deblocking   Deblock::strength deblock.cc:236-289 (4:2:2 keeps the four horizontal chroma
//                edges, :273-274), filter_edge :418-486 (chroma edge e reads strength_hor[e] and
//                the bS of luma column 2 x, :433 / :455), the chroma filter :380-400.
// Two places where the restatement has to choose (oracle/h264r_oracle.c, same choices):
//   - the chroma DC dequantisation uses qp_scaled[pl] as the reference does; 8.5.11.2 adds 3
//     (QP'c,DC = QP'c + 3), which the reference's author dropped on purpose
//     (R/doc/bugs-jm-18.5.txt item 11).  Results equal the reference's.
//   - an MB with transform_size_8x8_flag has no luma bS for its horizontal edges 1 and 3 in the
//     reference (strength_horizontal runs for filtered luma edges only, :280-285), yet filter_edge
//     reads them for the chroma edges at rows 4 and 12: the reference takes whatever the mb_t
//     slot last held.  These kernels derive them as 8.7.2.1 and JM do (intra 3; a coded 8x8
//     block 2; else 0, the two sides sharing one 8x8 partition).
//
// Schedule: an MB is one wave (64 lanes: lane = plane << 5 | 4x4 block << 2 | row).  Inter and
// PCM MBs need nothing of the picture: one launch takes them all.  Intra prediction reads the
// left, upper and upper-left MBs' unfiltered samples, and deblocking filters MB (x, y) after
// MB (x + 1, y - 1) (the raster order's result, mb_deblock.h): those two walk the picture with one
// workgroup of C422_WAVES waves per picture, wave w taking MB rows w, w + C422_WAVES, ..., with
// per-row progress in LDS.  Every wait is bounded (WaitClock).
#include "device_common.h"
#include "mb_deblock.h"

namespace h264r {

constexpr int C422_WAVES = 16;
constexpr int C422_MAX_ROWS = 1024;         // the context's max_height_mbs bound (h264r_create)

struct C422Wave {
    int nb[2][28];          // per plane: [0..15] p(-1, y), [16..23] p(x, -1), [24] p(-1, -1)
    int res[2][16][8];      // lossless residual before its DPCM
};

DEV int c422_rshift_rnd(int x, int a) { return a > 0 ? (x + (1 << (a - 1))) >> a : x * (1 << -a); }   // inter_prediction.cc:35-38

DEV int c422_tab_plane_offset(const h264r_batch& b, int pic) { return b.ref_planes_stride ? pic : 0; }

// One MB's 8 x 16 samples of both chroma planes.  Lane: plane p, 4x4 block blk (bx = blk & 1,
// by = blk >> 1), row r of the block: the 4 samples of chroma row 4 by + r, columns 4 bx ...
DEV void c422_mb(const h264r_batch& b, const Geom& g, int pic, int addr, int lane, C422Wave& S, const h264r_mb& m,
                 int cip, int* err)
{
    const int p = lane >> 5, blk = (lane >> 2) & 7, r = lane & 3;
    const int bx = blk & 1, by = blk >> 1;
    const int y = by * 4 + r, x0 = bx * 4;
    const int mbx = addr % g.wmb, mby = addr / g.wmb;
    const int Wc = g.Wc, Hc = g.hmb * 16;
    uint8_t* plane = (p ? b.out_v : b.out_u) + (size_t)pic * Wc * Hc;
    uint8_t* dst = plane + (size_t)(mby * 16 + y) * Wc + mbx * 8 + x0;
    const int16_t* lv = b.levels + m.coef_off;

    if (m.mb_type == H264R_I_PCM) {                 // Y 256, Cb 128, Cr 128 bytes (include/h264r.h)
        const uint8_t* raw = reinterpret_cast<const uint8_t*>(lv) + 256 + p * 128 + y * 8 + x0;
        *reinterpret_cast<uint32_t*>(dst) = *reinterpret_cast<const uint32_t*>(raw);
        return;
    }
    const int cbpl = m.cbp & 15, cbpc = m.cbp >> 4;
    const int intra = mb_is_intra(m), bypass = (m.flags & H264R_MBF_BYPASS) != 0;

    // ---- residual (the 4:2:2 level block: luma, then chroma AC 2 x 8 x 16, then DC 2 x 8)
    int res[4] = {0, 0, 0, 0};
    if (cbpc) {
        const int lumalen = 64 * __builtin_popcount(cbpl) + (m.mb_type == H264R_I_16x16 ? 16 : 0);
        int lev[4] = {0, 0, 0, 0};
        if (cbpc == 2) {
            const int16_t* a = lv + lumalen + p * 128 + blk * 16 + r * 4;
#pragma unroll
            for (int k = 0; k < 4; ++k) lev[k] = a[k];
        }
        const int16_t* dc = lv + lumalen + (cbpc == 2 ? 256 : 0) + p * 8;
        if (bypass) {
            // levels are the residual (transform.cc:453-455; transform_chroma_dc does nothing, :860),
            // the DC at (0, 0) of its block
            if (r == 0) lev[0] = dc[by * 2 + bx];
#pragma unroll
            for (int k = 0; k < 4; ++k) S.res[p][y][x0 + k] = lev[k];
            wave_sync();
            const int mode = m.chroma_mode;             // bypass_chroma: 2 vertical, 1 horizontal DPCM
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                int v = 0;
                if (mode == 2) { for (int yy = 0; yy <= y; ++yy) v += S.res[p][yy][x0 + k]; }
                else if (mode == 1) { for (int xx = 0; xx <= x0 + k; ++xx) v += S.res[p][y][xx]; }
                else v = S.res[p][y][x0 + k];
                res[k] = v;
            }
            wave_sync();
        } else {
            const int qP = m.qp_scaled[1 + p], per = qP / 6;
            const int16_t* sc = b.quant[pic].scale4x4[intra ? 0 : 1][1 + p][qP % 6];
            int d[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = lev[k] ? dq4(lev[k], sc[r * 4 + k], per) : 0;
            if (r == 0) {
                // transform_chroma_dc, ChromaArrayType 2: ihadamard_2x4 of the raster 2x4 DC matrix
                int c[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) c[k] = dc[k];
                int e[4][2], f[4][2];
#pragma unroll
                for (int i = 0; i < 4; ++i) { e[i][0] = c[2 * i] + c[2 * i + 1]; e[i][1] = c[2 * i] - c[2 * i + 1]; }
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int h0 = e[0][j] + e[2][j], h1 = e[0][j] - e[2][j], h2 = e[1][j] - e[3][j], h3 = e[1][j] + e[3][j];
                    f[0][j] = h0 + h3; f[1][j] = h1 + h2; f[2][j] = h1 - h2; f[3][j] = h0 - h3;
                }
                int fv = 0;                          // f[by][bx] by selects (no indexed registers)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) fv = (i == by && j == bx) ? f[i][j] : fv;
                const int v = fv * sc[0];
                d[0] = qP >= 36 ? v * (1 << (qP / 6 - 6)) : (v + (1 << (5 - qP / 6))) >> (6 - qP / 6);
            }
            int t[4];
            idct4(d[0], d[1], d[2], d[3], t[0], t[1], t[2], t[3]);          // my row
            const int q0 = lane & ~3;
#pragma unroll
            for (int j = 0; j < 4; ++j) {                                    // column j across the block's rows
                const int c0 = __shfl(t[j], q0 + 0), c1 = __shfl(t[j], q0 + 1);
                const int c2 = __shfl(t[j], q0 + 2), c3 = __shfl(t[j], q0 + 3);
                res[j] = idct4_col_row(c0, c1, c2, c3, r);
            }
        }
    }

    // ---- prediction
    int pred[4];
    if (intra) {
        const h264r_mb* mbs = b.mbs + (size_t)pic * g.nmb;
        auto avail = [&](int nx, int ny) {
            if (nx < 0 || ny < 0) return 0;
            const h264r_mb n = load_mb_const(mbs + ny * g.wmb + nx);
            return (int)(n.slice == m.slice && (!cip || mb_is_intra(n)));
        };
        const int avA = avail(mbx - 1, mby), avB = avail(mbx, mby - 1), avD = avail(mbx - 1, mby - 1);
        const int k = lane & 31;
        if (k < 25) {
            int v = 0;
            const int X = mbx * 8, Y = mby * 16;
            if (k < 16) { if (avA) v = plane[(size_t)(Y + k) * Wc + X - 1]; }
            else if (k < 24) { if (avB) v = plane[(size_t)(Y - 1) * Wc + X + k - 16]; }
            else if (avD) v = plane[(size_t)(Y - 1) * Wc + X - 1];
            S.nb[p][k] = v;
        }
        wave_sync();
        const int* L = S.nb[p];          // L[y] = p(-1, y); L[16 + x] = p(x, -1); L[24] = p(-1, -1)
        const int mode = m.chroma_mode;
        if (mode == 0) {                 // DC per 4x4 block (:825-849)
            const int xO = x0, yO = by * 4;
            int aA, aB;
            if ((xO == 0 && yO == 0) || (xO > 0 && yO > 0)) { aA = avA; aB = avB; }
            else if (xO > 0 && yO == 0) { aA = avB ? 0 : avA; aB = avB; }
            else { aA = avA; aB = avA ? 0 : avB; }
            int s = 0, v = 128;
            if (aA || aB) {
                if (aA) for (int i = 0; i < 4; ++i) s += L[yO + i];
                if (aB) for (int i = 0; i < 4; ++i) s += L[16 + xO + i];
                v = (s + (aA ? 2 : 0) + (aB ? 2 : 0)) >> (1 + aA + aB);
            }
            for (int i = 0; i < 4; ++i) pred[i] = v;
        } else if (mode == 1) {
            for (int i = 0; i < 4; ++i) pred[i] = L[y];
        } else if (mode == 2) {
            for (int i = 0; i < 4; ++i) pred[i] = L[16 + x0 + i];
        } else {                         // plane, yCF 4 (:871-894)
            auto top = [&](int x) { return x < 0 ? L[24] : L[16 + x]; };
            auto left = [&](int yy) { return yy < 0 ? L[24] : L[yy]; };
            int H = 0, V = 0;
            for (int i = 0; i < 4; ++i) H += (i + 1) * (top(4 + i) - top(2 - i));
            for (int i = 0; i < 8; ++i) V += (i + 1) * (left(8 + i) - left(6 - i));
            const int a = 16 * (L[15] + L[23]), bb = (34 * H + 32) >> 6, cc = (5 * V + 32) >> 6;
            for (int i = 0; i < 4; ++i) pred[i] = clip255((a + bb * (x0 + i - 3) + cc * (y - 7) + 16) >> 5);
        }
        wave_sync();                     // S.nb is rewritten by the next intra MB
    } else {
        // per 4x4 luma block: chroma columns 4 bx + {0,1} belong to luma block 2 bx, {2,3} to 2 bx + 1
        const h264r_slice* sl = b.slices + (size_t)pic * b.slice_stride + m.slice;
        const uint8_t* const* tab = b.ref_planes + (size_t)c422_tab_plane_offset(b, pic) * b.ref_planes_stride;
        const size_t mp = (size_t)g.motion_plane;
        const uint32_t* mvp = b.mv + (size_t)pic * 2 * mp;
        const int8_t* rip = b.ref_idx + (size_t)pic * 2 * mp;
        const int wpm = sl->wp_mode, lwd = sl->chroma_log2_wd;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int i4 = 2 * bx + h, j4 = by;
            const size_t idx = (size_t)(mby * 4 + j4) * g.W4 + mbx * 4 + i4;
            int ri[2], v[2][2] = {{0, 0}, {0, 0}};
#pragma unroll
            for (int l = 0; l < 2; ++l) {
                ri[l] = rip[l * mp + idx];
                if (ri[l] < 0) continue;
                const uint32_t mv = mvp[l * mp + idx];
                const int mvx = (int16_t)(mv & 0xFFFF), mvy = (int16_t)(mv >> 16);
                const int slot = sl->ref_slot[l][ri[l] & 15];
                const uint8_t* ref = (slot >= 0 && slot < H264R_MAX_SLOTS) ? tab[3 * slot + 1 + p] : nullptr;
                if (!ref) { __hip_atomic_store(err, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); continue; }
                const int xf = mvx & 7, yf = (mvy & 3) << 1;
                const int yi = mby * 16 + y + (mvy >> 2);
                const int y0c = clip3(0, Hc - 1, yi), y1c = clip3(0, Hc - 1, yi + 1);
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const int xi = mbx * 8 + x0 + 2 * h + s + (mvx >> 3);
                    const int xa = clip3(0, Wc - 1, xi), xb = clip3(0, Wc - 1, xi + 1);
                    const int A = ref[(size_t)y0c * Wc + xa], B = ref[(size_t)y0c * Wc + xb];
                    const int C = ref[(size_t)y1c * Wc + xa], D = ref[(size_t)y1c * Wc + xb];
                    v[l][s] = ((8 - xf) * (8 - yf) * A + xf * (8 - yf) * B + (8 - xf) * yf * C + xf * yf * D + 32) >> 6;
                }
            }
            const int dir = ri[0] >= 0 && ri[1] >= 0 ? 2 : ri[0] >= 0 ? 0 : 1;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                int o;
                if (dir != 2) {
                    const int vd = dir ? v[1][s] : v[0][s], rd = (dir ? ri[1] : ri[0]) & 15;
                    if (wpm == 1) {           // mc_prediction :62-85
                        const int w = sl->wp_weight[dir][rd][1 + p], off = sl->wp_offset[dir][rd][1 + p];
                        o = clip255(c422_rshift_rnd(w * vd, lwd) + off);
                    } else o = vd;
                } else if (wpm) {             // bi_prediction :99-153
                    int w0, w1, o0, o1;
                    if (wpm == 1) {
                        w0 = sl->wp_weight[0][ri[0] & 15][1 + p]; w1 = sl->wp_weight[1][ri[1] & 15][1 + p];
                        o0 = sl->wp_offset[0][ri[0] & 15][1 + p]; o1 = sl->wp_offset[1][ri[1] & 15][1 + p];
                    } else {
                        w1 = sl->implicit_w1[ri[0] & 15][ri[1] & 15]; w0 = 64 - w1; o0 = o1 = 0;
                    }
                    o = clip255(c422_rshift_rnd(w0 * v[0][s] + w1 * v[1][s], lwd + 1) + ((o0 + o1 + 1) >> 1));
                } else o = (v[0][s] + v[1][s] + 1) >> 1;
                pred[2 * h + s] = o;
            }
        }
    }
    uint32_t w = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) w |= (uint32_t)clip255(pred[k] + res[k]) << (8 * k);
    *reinterpret_cast<uint32_t*>(dst) = w;
}

// Inter and I_PCM MBs read nothing of the picture being decoded: k_c422_inter reconstructs them
// all at once, one wave per MB (grid: ceil(pictures x band MBs / 4) workgroups of 4 waves).
extern "C" __global__ __launch_bounds__(256) void k_c422_inter(h264r_batch b, int2 rows, int* err)
{
    __shared__ C422Wave ws[4];
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nband = (rows.y - rows.x) * g.wmb;
    const int64_t t = (int64_t)blockIdx.x * 4 + wave;
    if (t >= (int64_t)b.num_pics * nband) return;
    const int pic = (int)(t / nband), addr = rows.x * g.wmb + (int)(t % nband);
    const h264r_mb m = load_mb_const(b.mbs + (size_t)pic * g.nmb + addr);
    if (mb_is_intra(m) && m.mb_type != H264R_I_PCM) return;              // k_c422_intra
    if ((ld_const(&b.slices[(size_t)pic * b.slice_stride + m.slice]) & 255) == H264R_SLICE_SP && lane == 0)
        __hip_atomic_store(err, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // SP is 4:2:0 only
    c422_mb(b, g, pic, addr, lane, ws[wave], m, 0, err);
}

// The intra MBs (not I_PCM), after k_c422_inter: one workgroup of C422_WAVES waves per picture,
// wave w walks MB rows w, w + C422_WAVES, ... of the band [rows.x, rows.y), skipping the other
// MBs.  Before an intra MB at column x waits for the row above to pass x (its upper and
// upper-left neighbours), it publishes x for the row below (every MB left of it is done).
extern "C" __global__ __launch_bounds__(64 * C422_WAVES) void k_c422_intra(h264r_batch b, int2 rows, int* err)
{
    __shared__ int prog[C422_MAX_ROWS];
    __shared__ C422Wave ws[C422_WAVES];
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int pic = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < rows.y - rows.x; i += blockDim.x) prog[i] = 0;
    __syncthreads();
    const int cip = (int)__builtin_amdgcn_readfirstlane(ld_const(&b.pics[pic].constrained_intra_pred));
    auto publish = [&](int ri, int v) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_store(&prog[ri], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    for (int row = rows.x + wave; row < rows.y; row += C422_WAVES) {
        const int ri = row - rows.x;
        WaitClock wc;
        // the row's intra MBs 64 columns at a time: one record word per lane, a ballot
        for (int xb = 0; xb < g.wmb; xb += 64) {
            const int xl = xb + lane;
            int is = 0;
            if (xl < g.wmb) {
                const uint32_t w0 = *reinterpret_cast<const uint32_t*>(b.mbs + (size_t)pic * g.nmb + row * g.wmb + xl);
                is = ((w0 >> 8) & H264R_MBF_INTRA) && (w0 & 255) != H264R_I_PCM;        // flags, mb_type
            }
            uint64_t mask = __ballot(is);
            while (mask) {
            const int x = xb + __builtin_ctzll(mask);
            mask &= mask - 1;
            const int addr = row * g.wmb + x;
            const h264r_mb m = load_mb_const(b.mbs + (size_t)pic * g.nmb + addr);
            publish(ri, x);
            if (ri > 0) {
                while (__hip_atomic_load(&prog[ri - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <= x) {
                    if (wait_give_up(err, wc)) return;
                    __builtin_amdgcn_s_sleep(1);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
            c422_mb(b, g, pic, addr, lane, ws[wave], m, cip, err);
            }
        }
        publish(ri, g.wmb);
    }
}

// ------------------------------------------------------------------------------ deblocking
struct C422DbWave {
    uint8_t t[2][18][12];    // per plane: rows -2..15, columns -2..7 of the MB (index + 2)
    uint32_t info[DBINFO_DWORDS];
    uint32_t rec[8];         // the MB's h264r_mb
};

// the chroma filter of filter_edge (chromaStyleFilteringFlag, deblock.cc:350-364, 380-400):
// p0 / q0 only; w = edge_word() (alpha | beta << 8 | tc0 of bS 1..3 from bit 16, 5 bits each)
DEV void c422_filter(uint8_t* p1, uint8_t* p0, uint8_t* q0, uint8_t* q1, int bs, uint32_t w)
{
    const int alpha = w & 255, beta = (w >> 8) & 255;
    const int P1 = *p1, P0 = *p0, Q0 = *q0, Q1 = *q1;
    if (!(iabs(P0 - Q0) < alpha && iabs(P1 - P0) < beta && iabs(Q1 - Q0) < beta)) return;
    if (bs == 4) {
        *p0 = (uint8_t)((2 * P1 + P0 + Q1 + 2) >> 2);
        *q0 = (uint8_t)((2 * Q1 + Q0 + P1 + 2) >> 2);
    } else {
        const int tc = (int)((w >> (16 + 5 * (bs - 1))) & 31) + 1;
        const int delta = clip3(-tc, tc, (((Q0 - P0) * 4) + (P1 - Q1) + 4) >> 3);
        *p0 = (uint8_t)clip255(P0 + delta);
        *q0 = (uint8_t)clip255(Q0 - delta);
    }
}

// The MB-row walk of the deblocking: MB x's rows 0..15 (columns 0..7), its deblocking record and
// its MB record are prefetched two MBs ahead (nothing but MB x itself changes those rows before it
// is filtered: the row below touches MB x only after this row has passed x + 1); its columns
// -2, -1 are MB x - 1's final columns 6, 7, kept in the tile; rows -2, -1 come from the row above
// after the wait.  The stores of MB x are waited for one MB later, when MB x + 1 publishes.
struct C422DbPrefetch {
    uint2 row;          // lanes 0..31: plane lane >> 4, row lane & 15, columns 0..7
    uint32_t info;      // lanes 32..51: DbInfo dword lane - 32; lanes 52..59: h264r_mb dword lane - 52
};

DEV C422DbPrefetch c422_db_prefetch(const h264r_batch& b, const Geom& g, uint8_t* const (&planes)[2],
                                    const DbInfo* __restrict__ dbinfo, int pic, int addr, int lane)
{
    C422DbPrefetch f;
    f.row = make_uint2(0, 0); f.info = 0;
    const int mbx = addr % g.wmb, mby = addr / g.wmb;
    if (lane < 32)
        f.row = *reinterpret_cast<const uint2*>(planes[lane >> 4] + (size_t)(mby * 16 + (lane & 15)) * g.Wc + mbx * 8);
    else if (lane < 32 + DBINFO_DWORDS)
        f.info = reinterpret_cast<const uint32_t*>(dbinfo + (size_t)pic * g.nmb + addr)[lane - 32];
    else if (lane < 60)
        f.info = reinterpret_cast<const uint32_t*>(b.mbs + (size_t)pic * g.nmb + addr)[lane - 52];
    return f;
}

DEV void c422_put8(uint8_t* t, uint2 v)
{
#pragma unroll
    for (int k = 0; k < 4; ++k) { t[k] = (uint8_t)(v.x >> (8 * k)); t[4 + k] = (uint8_t)(v.y >> (8 * k)); }
}
DEV uint2 c422_get8(const uint8_t* s)
{
    return make_uint2(s[0] | (s[1] << 8) | (s[2] << 16) | ((uint32_t)s[3] << 24),
                      s[4] | (s[5] << 8) | (s[6] << 16) | ((uint32_t)s[7] << 24));
}

// Grid: one workgroup per picture, C422_WAVES waves; dbinfo: the luma pass's records
// (pic * W * H + addr).  MB (x, y) waits for MB (x + 1, y - 1) of the band.
extern "C" __global__ __launch_bounds__(64 * C422_WAVES) void k_c422_db(h264r_batch b, const DbInfo* __restrict__ dbinfo,
                                                                        int2 rows, int* err)
{
    __shared__ int prog[C422_MAX_ROWS];
    __shared__ C422DbWave ws[C422_WAVES];
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int pic = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int Wc = g.Wc, Hc = g.hmb * 16;
    uint8_t* const planes[2] = {b.out_u + (size_t)pic * Wc * Hc, b.out_v + (size_t)pic * Wc * Hc};
    C422DbWave& T = ws[wave];
    for (int i = threadIdx.x; i < rows.y - rows.x; i += blockDim.x) prog[i] = 0;
    __syncthreads();
    auto publish = [&](int ri, int v) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_store(&prog[ri], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    for (int row = rows.x + wave; row < rows.y; row += C422_WAVES) {
        const int ri = row - rows.x, Y = row * 16;
        WaitClock wc;
        C422DbPrefetch f = c422_db_prefetch(b, g, planes, dbinfo, pic, row * g.wmb, lane);
        C422DbPrefetch f2 = f;
        if (g.wmb > 1) f2 = c422_db_prefetch(b, g, planes, dbinfo, pic, row * g.wmb + 1, lane);
        for (int x = 0; x < g.wmb; ++x) {
            const int addr = row * g.wmb + x, X = x * 8;
            // the tile: columns -2, -1 = MB x - 1's columns 6, 7 (same lane, read before the write)
            if (lane < 32) {
                uint8_t* t = &T.t[lane >> 4][(lane & 15) + 2][0];
                t[0] = t[8]; t[1] = t[9];
                c422_put8(t + 2, f.row);
            } else if (lane < 32 + DBINFO_DWORDS) {
                T.info[lane - 32] = f.info;
            } else if (lane < 60) {
                T.rec[lane - 52] = f.info;
            }
            f = f2;
            if (ri > 0) {
                const int need = min(x + 2, g.wmb);
                while (__hip_atomic_load(&prog[ri - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
                    if (wait_give_up(err, wc)) return;
                    __builtin_amdgcn_s_sleep(1);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
            if (lane >= 60 && Y > 0) {                        // rows -2, -1 of both planes, columns 0..7
                const int q = lane - 60, p = q >> 1, k = q & 1;
                c422_put8(&T.t[p][k][2], *reinterpret_cast<const uint2*>(planes[p] + (size_t)(Y - 2 + k) * Wc + X));
            }
            wave_sync();
            h264r_mb m;
            {
                uint32_t* w = reinterpret_cast<uint32_t*>(&m);
#pragma unroll
                for (int k = 0; k < 8; ++k) w[k] = T.rec[k];
            }
            const uint8_t* bsv = reinterpret_cast<const uint8_t*>(T.info);       // DbInfo::bs
            const uint32_t* par = T.info + 8;                                     // DbInfo::par
            {   // vertical edges 0 and 1 (chroma columns 0, 4: luma edges 0, 2), rows 0..15
                const int p = lane >> 5, e = (lane >> 4) & 1, yr = lane & 15;
                const int bs = bsv[(2 * e) * 4 + (yr >> 2)];
                if (bs) {
                    uint8_t* q = &T.t[p][yr + 2][2 + 4 * e];
                    c422_filter(q - 2, q - 1, q, q + 1, bs, par[3 + 3 * p + (e ? 2 : 0)]);
                }
            }
            wave_sync();
            {   // horizontal edges 0..3 (chroma rows 0, 4, 8, 12 -- strength_hor[e], luma column 2 x)
                const int p = lane >> 5, e = (lane >> 3) & 3, xc = lane & 7;
                int bs = bsv[16 + e * 4 + (xc >> 1)];
                if ((e & 1) && (m.flags & H264R_MBF_T8x8)) {
                    // no luma edge here: 8.7.2.1 / JM (the file comment)
                    const int idc = (int)((ld_const(&b.slices[(size_t)pic * b.slice_stride + m.slice]) >> 8) & 255);
                    bs = idc == 1 ? 0 : mb_is_intra(m) ? 3 : ((m.cbp_blks >> (4 * e + (xc >> 1))) & 1) ? 2 : 0;
                }
                if (bs) {
                    uint8_t* q = &T.t[p][4 * e + 2][2 + xc];
                    constexpr int S = 12;
                    c422_filter(q - 2 * S, q - S, q, q + S, bs, par[3 + 3 * p + (e ? 2 : 1)]);
                }
            }
            wave_sync();
            publish(ri, x);                                    // MB x - 1's stores are done
            if (lane < 32) {                                   // rows 0..15: columns 0..7, and -1
                const int p = lane >> 4, yr = lane & 15;
                uint8_t* dst = planes[p] + (size_t)(Y + yr) * Wc + X;
                const uint8_t* s = &T.t[p][yr + 2][2];
                *reinterpret_cast<uint2*>(dst) = c422_get8(s);
                if (X > 0) dst[-1] = s[-1];
            } else if (lane < 34 && ri > 0 && Y > 0) {        // row -1 (the top edge's p0)
                const int p = lane - 32;
                *reinterpret_cast<uint2*>(planes[p] + (size_t)(Y - 1) * Wc + X) = c422_get8(&T.t[p][1][2]);
            }
            if (x + 2 < g.wmb) f2 = c422_db_prefetch(b, g, planes, dbinfo, pic, addr + 2, lane);
            wave_sync();                                       // the tile is rewritten by MB x + 1
        }
        publish(ri, g.wmb);
    }
}

}  // namespace h264r
