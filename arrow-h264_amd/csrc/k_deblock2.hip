// k_deblock2.hip -- the in-loop deblocking filter for large batches: register-resident
// MB walks, a lane pair per (picture, MB row), packed 16-bit filters.
//
// The reference filters MB by MB in raster order, vertical edges then horizontal edges
// (Deblock::deblock_pic, deblock.cc:537-552): along a row MB x needs MB x-1 finished,
// and MB (x, y) needs MB (x+1, y-1) finished -- a wavefront with a 2-MB lag per row.
// k_deblock (k_deblock.hip) spreads one MB over 32 lanes and exchanges every line through
// LDS; its steps are short but latency-bound.  Here the parallelism comes from the
// pictures of the batch instead: one 64-lane wave owns MB row y of 32 pictures, two lanes
// per picture ("unit"), and walks x = 0 .. W-1 with every unit in lock step.  A lane keeps
// its half of the MB in registers for the whole step:
//
//   vertical edges   lane h filters luma rows 8h .. 8h+7 and chroma plane h (Cb / Cr),
//                    rows paired (r, r+4) in s16x2 -- filter_vertical deblock.cc:488-504
//   horizontal edges lane h filters luma columns 8h .. 8h+7 and chroma plane h, columns
//                    paired (c, c+4) -- filter_horizontal :506-535; the luma half-MBs are
//                    swapped between the two lanes of the unit with one DPP move each
//
// The rows below need each MB's bottom rows after the MB's right neighbour filtered its
// left edge: the record of MB x-1 (luma rows 12..15, chroma rows 6..7, the lane's half)
// is published at step x as 12 naturally aligned 8-byte granules {data dword, launch
// epoch} (write-through `sc1` stores), and the row below re-polls them with `sc1` loads
// until every granule carries this launch's epoch (MI355X_MICROARCH.md R2 granule
// hand-off).  Waves take tickets row-major, so a wave only waits on tickets taken earlier
// by running waves; every spin is bounded and flags the error word.
//
// Sample ownership (each sample stored once, when final): a row stores, at step x, the
// luma rows 0..12 (chroma 0..6) of MB x except the columns MB x+1's left edge still
// changes (luma 12..15, chroma 4..7: stored at step x+1, or at the row end), and the
// rows 13..15 (chroma 7) of MB (x, y-1) after filtering its own top edge.  The last row
// of the band stores its own bottom rows.
#include "mb_deblock.h"
#include "mb_deblock2.h"

using namespace h264r;

namespace {

constexpr unsigned SPIN2 = 1u << 22;   // bounded polling, then flag an error
constexpr int RECN = 12;               // granules per lane per record

DEV uint64_t ldcc64(const uint64_t* p) { return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DEV void stcc64(uint64_t* p, uint64_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DEV uint32_t swap_pair(uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false); }  // lane ^ 1

template <typename T>
DEV T gld(const void* p) { return *(const T*)p; }
template <typename T>
DEV void gst(void* p, T v) { *(T*)p = v; }

}  // namespace

// hb: records [pic][row & 1][W][2][RECN] granules {dword, tag}; sync[0]: ticket counter;
// epoch < 2^20 (the host restarts from zeroed records before it wraps).
extern "C" __global__ __launch_bounds__(64) void k_deblock2(h264r_batch b, const DbInfo* __restrict__ dbinfo, uint64_t* hb,
                                                            int* sync, int* err, uint32_t epoch, int2 rows)
{
    const int lane = threadIdx.x, h = lane & 1, u = lane >> 1;
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int W = g.wmb, R0 = rows.x, R1 = rows.y;
    const int ngroups = (b.num_pics + 31) >> 5;
    int tk = 0;
    if (lane == 0) tk = atomicAdd(&sync[0], 1);
    const int ticket = __builtin_amdgcn_readfirstlane(tk);
    const int ry = ticket / ngroups, grp = ticket - ry * ngroups;
    const int y = R0 + ry;
    const int pic_raw = grp * 32 + u;
    const bool active = pic_raw < b.num_pics;
    const int pic = active ? pic_raw : b.num_pics - 1;
    const bool above = y > R0, last_row = y == R1 - 1;
    // records live in two slots per picture (rows alternate); the tag names launch and row
    const uint64_t tag = (uint64_t)((epoch << 12) | ((uint32_t)ry & 0xFFFu)) << 32;
    const uint64_t tag_in = (uint64_t)((epoch << 12) | ((uint32_t)(ry - 1) & 0xFFFu)) << 32;

    uint8_t* Y = b.out_y + (size_t)pic * g.ysz;
    uint8_t* C = (h ? b.out_v : b.out_u) + (size_t)pic * g.csz;
    const size_t Wl = (size_t)g.W, Wc = (size_t)g.Wc;
    uint8_t* yrow = Y + (size_t)(y * 16 + 8 * h) * Wl;          // my first V row (luma)
    uint8_t* crow = C + (size_t)(y * 8) * Wc;                   // my plane's MB row (chroma)
    const uint32_t* info_row = reinterpret_cast<const uint32_t*>(dbinfo + (size_t)pic * g.nmb + (size_t)y * W);
    uint64_t* rec_out = hb + (((size_t)pic * 2 + (ry & 1)) * W) * (2 * RECN) + h * RECN;
    const uint64_t* rec_in = above ? hb + (((size_t)pic * 2 + ((ry - 1) & 1)) * W) * (2 * RECN) + h * RECN : rec_out;

    // ---- per-step inputs, prefetched one step ahead
    uint32_t R[8][4];          // luma rows 8h .. 8h+7 of MB x
    uint32_t CR[8][2];         // chroma plane h rows 0..7 of MB x
    uint32_t inf[20];          // DbInfo of MB x
    uint64_t rin[RECN];        // record of MB (x, y-1) from the row above (my half)
    uint32_t nR[8][4], nCR[8][2], ninf[20];
    auto load_rec = [&](int x) {
#pragma unroll
        for (int k = 0; k < RECN; ++k) rin[k] = ldcc64(rec_in + (size_t)x * (2 * RECN) + k);
    };
    auto load_mb = [&](int x, uint32_t (&r)[8][4], uint32_t (&c)[8][2], uint32_t (&in)[20]) {
        const int xs = min(x, W - 1);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint4 v = gld<uint4>(yrow + (size_t)i * Wl + xs * 16);
            r[i][0] = v.x; r[i][1] = v.y; r[i][2] = v.z; r[i][3] = v.w;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint2 v = gld<uint2>(crow + (size_t)i * Wc + xs * 8);
            c[i][0] = v.x; c[i][1] = v.y;
        }
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint4 v = gld<uint4>(info_row + (size_t)xs * DBINFO_DWORDS + 4 * k);
            in[4 * k] = v.x; in[4 * k + 1] = v.y; in[4 * k + 2] = v.z; in[4 * k + 3] = v.w;
        }
    };

    // ---- loop-carried state
    uint32_t lf[8];            // luma cols 12..15 of MB x-1, my V rows (after H(x-1))
    uint32_t cl[8];            // chroma cols 4..7 of MB x-1, rows 0..7 (after H(x-1))
    uint32_t rc_l[4][2];       // luma rows 12..15 of MB x-1, my H columns (after H(x-1))
    uint32_t rc_c[2];          // chroma rows 6..7 cols 0..3 of MB x-1 (after H(x-1))
#pragma unroll
    for (int i = 0; i < 8; ++i) lf[i] = cl[i] = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) rc_l[i][0] = rc_l[i][1] = 0;
    rc_c[0] = rc_c[1] = 0;
    bool ok = true;

    load_mb(0, R, CR, inf);
    for (int x = 0; x <= W; ++x) {
        const bool cur = x < W;
        if (cur && above) load_rec(x);           // polled after the vertical edges
        if (x + 1 < W) load_mb(x + 1, nR, nCR, ninf);

        // ================= vertical edges of MB x (deblock.cc:488-504)
        if (cur) {
            // luma: rows (8h + i, 8h + i + 4); bS of V edge e, segment s: byte 4e + s
            EdgeP ev[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const s2 bsx = (s2){(short)((inf[e] >> (16 * h)) & 255), (short)((inf[e] >> (16 * h + 8)) & 255)};
                ev[e] = edge_params(inf[8 + (e == 0 ? 0 : 2)], bsx);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                s2 c[20];
                c[0] = unpack2(lf[i], lf[i + 4], 0); c[1] = unpack2(lf[i], lf[i + 4], 1);
                c[2] = unpack2(lf[i], lf[i + 4], 2); c[3] = unpack2(lf[i], lf[i + 4], 3);
#pragma unroll
                for (int k = 4; k < 20; ++k) c[k] = unpack2(R[i][(k >> 2) - 1], R[i + 4][(k >> 2) - 1], k & 3);
                filter2<true, false>(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], ev[0]);
#pragma unroll
                for (int e = 1; e < 4; ++e)
                    filter2<false, false>(c[4 * e], c[4 * e + 1], c[4 * e + 2], c[4 * e + 3], c[4 * e + 4], c[4 * e + 5],
                                          c[4 * e + 6], c[4 * e + 7], ev[e]);
                pack4(c[0], c[1], c[2], c[3], lf[i], lf[i + 4]);
#pragma unroll
                for (int d = 0; d < 4; ++d) pack4(c[4 + 4 * d], c[5 + 4 * d], c[6 + 4 * d], c[7 + 4 * d], R[i][d], R[i + 4][d]);
            }
            // chroma plane h: rows (i, i + 4); chroma edge 0 = luma edge 0, edge 1 (col 4) = luma
            // edge 2; row j takes the bS of luma row 2j (deblock.cc:430-433, 460): segment j / 2
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int s = i >> 1;
                EdgeP ec[2];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const uint32_t w = inf[e * 2];
                    const s2 bsx = (s2){(short)((w >> (8 * s)) & 255), (short)((w >> (8 * (s + 2))) & 255)};
                    ec[e] = edge_params(inf[8 + 3 * (1 + h) + (e == 0 ? 0 : 2)], bsx);
                }
                s2 c[12];
#pragma unroll
                for (int k = 0; k < 4; ++k) c[k] = unpack2(cl[i], cl[i + 4], k);
#pragma unroll
                for (int k = 4; k < 12; ++k) c[k] = unpack2(CR[i][(k >> 2) - 1], CR[i + 4][(k >> 2) - 1], k & 3);
                filter2<true, true>(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], ec[0]);
                filter2<false, true>(c[4], c[5], c[6], c[7], c[8], c[9], c[10], c[11], ec[1]);
                pack4(c[0], c[1], c[2], c[3], cl[i], cl[i + 4]);
                pack4(c[4], c[5], c[6], c[7], CR[i][0], CR[i + 4][0]);
                pack4(c[8], c[9], c[10], c[11], CR[i][1], CR[i + 4][1]);
            }
        }

        // ================= MB x-1 is final for this row: its record for the row below and
        // its columns MB x's left edge changed (luma 12..15, chroma 4..7)
        if (x >= 1) {
            if (!last_row && active) {
                // luma rows 12..15 of my H columns: cols 0..7 (lane 0) or 8..11 + 12..15 (lane 1;
                // cols 12..15 of rows 12..15 = lf[4..7] after V(x) -- or after H(W-1) at the end)
                uint64_t* dst = rec_out + (size_t)(x - 1) * (2 * RECN);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    stcc64(dst + 2 * i, tag | rc_l[i][0]);
                    stcc64(dst + 2 * i + 1, tag | (h ? lf[4 + i] : rc_l[i][1]));
                }
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    stcc64(dst + 8 + 2 * i, tag | rc_c[i]);
                    stcc64(dst + 9 + 2 * i, tag | cl[6 + i]);
                }
            }
            if (cur && active) {
                // luma cols 12..15 of MB x-1, my V rows (rows <= 12 unless last row)
                uint8_t* p = yrow + (x - 1) * 16 + 12;
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (8 * h + i <= 12 || last_row) gst<uint32_t>(p + (size_t)i * Wl, lf[i]);
                uint8_t* q = crow + (x - 1) * 8 + 4;
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (i <= 6 || last_row) gst<uint32_t>(q + (size_t)i * Wc, cl[i]);
            }
        }
        if (!cur) break;

        // ================= the record of MB (x, y-1) from the row above: wait for this epoch
        if (above) {
            unsigned spins = 0;
            for (;;) {
                bool ready = true;
#pragma unroll
                for (int k = 0; k < RECN; ++k) ready &= (rin[k] & 0xFFFFFFFF00000000ull) == tag_in;
                if (__all(ready || !active)) break;
                __builtin_amdgcn_s_sleep(1);
                load_rec(x);
                if (++spins > SPIN2) {
                    if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = false;
                    break;
                }
            }
            if (!ok) break;
        }

        // a band that starts below row 0 must not be filtered across its top edge (idc 1, or a
        // slice edge with idc 2): its top-edge strengths (bs[16..19] = info dword 4) are 0
        if (y == R0 && R0 > 0 && active && inf[4] != 0)
            __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

        // ================= horizontal edges of MB x (deblock.cc:506-535)
        // luma tile of my columns 8h .. 8h+7: T[r][j], r = -4..15 (index r + 4), j = dword
        uint32_t T[20][2];
#pragma unroll
        for (int i = 0; i < 4; ++i) { T[i][0] = (uint32_t)rin[2 * i]; T[i][1] = (uint32_t)rin[2 * i + 1]; }
        // my V rows hold dwords 2h, 2h+1 of my columns; the partner's rows arrive by DPP
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const uint32_t mine = h ? R[i][j + 2] : R[i][j];                 // my columns, my rows
                const uint32_t give = h ? R[i][j] : R[i][j + 2];                 // partner's columns, my rows
                const uint32_t got = swap_pair(give);                            // my columns, partner's rows
                T[4 + i][j] = h ? got : mine;                                    // rows 0..7
                T[12 + i][j] = h ? mine : got;                                   // rows 8..15
            }
        }
        {
            EdgeP eh[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t w = inf[4 + e];                                   // bs[16 + 4e + s]
                const s2 bsx = (s2){(short)((w >> (16 * h)) & 255), (short)((w >> (16 * h + 8)) & 255)};
                eh[e] = edge_params(inf[8 + (e == 0 ? 1 : 2)], bsx);
            }
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                s2 c[2][20];
#pragma unroll
                for (int b = 0; b < 2; ++b) {
#pragma unroll
                    for (int r = 0; r < 20; ++r) c[b][r] = unpack2(T[r][0], T[r][1], 2 * half + b);
                    filter2<true, false>(c[b][0], c[b][1], c[b][2], c[b][3], c[b][4], c[b][5], c[b][6], c[b][7], eh[0]);
#pragma unroll
                    for (int e = 1; e < 4; ++e)
                        filter2<false, false>(c[b][4 * e], c[b][4 * e + 1], c[b][4 * e + 2], c[b][4 * e + 3], c[b][4 * e + 4],
                                              c[b][4 * e + 5], c[b][4 * e + 6], c[b][4 * e + 7], eh[e]);
                }
#pragma unroll
                for (int r = 1; r < 20; ++r) merge2(c[0][r], c[1][r], half, T[r][0], T[r][1]);
            }
        }
        // chroma plane h, rows -2..7 (index r + 2), cols 0..7 as (b, b+4) pairs
        uint32_t TC[10][2];
        TC[0][0] = (uint32_t)rin[8]; TC[0][1] = (uint32_t)rin[9];
        TC[1][0] = (uint32_t)rin[10]; TC[1][1] = (uint32_t)rin[11];
#pragma unroll
        for (int i = 0; i < 8; ++i) { TC[2 + i][0] = CR[i][0]; TC[2 + i][1] = CR[i][1]; }
        {
            EdgeP eh[2][2];                                                      // [edge][segment pair]
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const uint32_t w = inf[4 + 2 * e];                               // chroma edge 1 = luma edge 2
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const s2 bsx = (s2){(short)((w >> (8 * s)) & 255), (short)((w >> (8 * (s + 2))) & 255)};
                    eh[e][s] = edge_params(inf[8 + 3 * (1 + h) + (e == 0 ? 1 : 2)], bsx);
                }
            }
            s2 c[4][10];
#pragma unroll
            for (int bcol = 0; bcol < 4; ++bcol) {
#pragma unroll
                for (int r = 0; r < 10; ++r) c[bcol][r] = unpack2(TC[r][0], TC[r][1], bcol);
                s2 d0 = c[bcol][0], d1 = c[bcol][9];
                filter2<true, true>(d0, d0, c[bcol][0], c[bcol][1], c[bcol][2], c[bcol][3], d1, d1, eh[0][bcol >> 1]);
                filter2<false, true>(d0, d0, c[bcol][4], c[bcol][5], c[bcol][6], c[bcol][7], d1, d1, eh[1][bcol >> 1]);
            }
#pragma unroll
            for (int r = 1; r < 8; ++r) pack4(c[0][r], c[1][r], c[2][r], c[3][r], TC[r][0], TC[r][1]);
        }

        // ================= stores of what is final now
        if (active) {
            // luma MB x rows 0..12 (0..15 in the last row), my columns except 12..15
            uint8_t* p = Y + (size_t)(y * 16) * Wl + x * 16 + 8 * h;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if (r > 12 && !last_row) continue;
                gst<uint32_t>(p + (size_t)r * Wl, T[4 + r][0]);
                if (!h || x == W - 1) gst<uint32_t>(p + (size_t)r * Wl + 4, T[4 + r][1]);
            }
            // rows 13..15 of MB (x, y-1), my columns
            if (above) {
#pragma unroll
                for (int r = 1; r < 4; ++r)
                    gst<uint2>(Y + (size_t)(y * 16 - 4 + r) * Wl + x * 16 + 8 * h, make_uint2(T[r][0], T[r][1]));
            }
            // chroma MB x rows 0..6 (0..7 in the last row), cols 0..3 (and 4..7 at the row end)
            uint8_t* q = crow + x * 8;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                if (r > 6 && !last_row) continue;
                gst<uint32_t>(q + (size_t)r * Wc, TC[2 + r][0]);
                if (x == W - 1) gst<uint32_t>(q + (size_t)r * Wc + 4, TC[2 + r][1]);
            }
            if (above) gst<uint2>(C + (size_t)(y * 8 - 1) * Wc + x * 8, make_uint2(TC[1][0], TC[1][1]));
        }

        // ================= carries for step x+1
        // left columns (cols 12..15 of MB x) of my V rows: rows 0..7 sit in lane 1's tile,
        // rows 8..15 in its own -- lane 0 receives them
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t give = T[4 + i][1];                                   // lane 1: rows 0..7, cols 12..15
            const uint32_t got = swap_pair(give);
            lf[i] = h ? T[12 + i][1] : got;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) cl[i] = TC[2 + i][1];
#pragma unroll
        for (int i = 0; i < 4; ++i) { rc_l[i][0] = T[16 + i][0]; rc_l[i][1] = T[16 + i][1]; }
        rc_c[0] = TC[8][0]; rc_c[1] = TC[9][0];

        // next MB
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#pragma unroll
            for (int j = 0; j < 4; ++j) R[i][j] = nR[i][j];
            CR[i][0] = nCR[i][0]; CR[i][1] = nCR[i][1];
        }
#pragma unroll
        for (int k = 0; k < 20; ++k) inf[k] = ninf[k];
    }
    if (!ok && !last_row)                        // release the row below (the error is flagged)
        for (int x = 0; x < W; ++x)
            for (int k = 0; k < RECN; ++k) stcc64(rec_out + (size_t)x * (2 * RECN) + k, tag);
}
