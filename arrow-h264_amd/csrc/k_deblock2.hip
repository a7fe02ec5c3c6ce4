// k_deblock2.hip -- the in-loop deblocking filter for large batches: MB-row walks of
// 16 pictures per wave, 4 lanes per (picture, MB row), packed 16-bit filters, LDS windows.
//
// The reference filters MB by MB in raster order, vertical edges then horizontal edges
// (Deblock::deblock_pic, deblock.cc:537-552): along a row MB x needs MB x-1 finished,
// and MB (x, y) needs MB (x+1, y-1) finished -- a wavefront with a 2-MB lag per row.
// k_deblock (k_deblock.hip) spreads one MB over 32 lanes; its steps are short but
// latency-bound.  Here the parallelism comes from the pictures of the batch: a 64-lane
// wave owns MB row y of 16 pictures, four lanes per picture ("unit"), and walks
// x = 0 .. W-1 with every unit in lock step.
//
//   vertical edges   lane q filters luma rows 4q .. 4q+3 as the pairs (r, r+2) and
//                    chroma plane q/2, rows 4(q&1) .. +3 -- filter_vertical deblock.cc:488-504
//   horizontal edges lane q filters luma columns 4q .. 4q+3 as the pairs (c, c+2) and
//                    chroma plane q/2, columns 4(q&1) .. +3 -- filter_horizontal :506-535
//
// Every operand is an s16x2 of two lines (mb_deblock2.h); the transposition between
// the two passes is free, since both read the MB from LDS.  Each unit's MB row lives
// in LDS as a ring of three MB slots (MB x in slot x % 3: the left neighbour stays
// while the next two MBs arrive); the two MBs of a window are fetched one window ahead
// into registers as 32-byte row pieces and written back as 16-byte pieces, so global
// traffic stays in whole sectors (a lane-pair walk with 16-byte scattered accesses
// missed L2: profiles/r02_deblock2_v1_pmc_b256.txt).
//
// The row below needs each MB's bottom rows (luma 12..15, chroma 6..7) after the
// MB's right neighbour filtered its left edge: 24 naturally aligned 8-byte granules
// {data dword, tag} per MB, 16 published after H(x) (the columns MB x+1 cannot
// change) and 8 after V(x+1) (luma columns 12..15, chroma 4..7), with write-through
// `sc1` stores; the row below re-polls them with `sc1` loads until every granule
// carries this launch's tag (MI355X_MICROARCH.md R2 granule hand-off).  Waves take
// tickets row-major, so a wave only waits on tickets taken earlier by running waves;
// every spin is bounded and flags the error word.
//
// Sample ownership (each sample stored once, when final): a row stores MB x's rows
// 0..12 (chroma 0..6) once MB x+1's vertical edges are done, and the rows 13..15
// (chroma 7) of MB (x, y-1) after filtering its own top edge.  The last row of the
// band stores its own bottom rows.
#include "mb_deblock.h"
#include "mb_deblock2.h"

using namespace h264r;

namespace {

constexpr unsigned SPIN2 = 1u << 22;   // bounded polling, then flag an error
constexpr int UNITS = DEBLOCK2_UNITS;  // (picture, MB row) units per wave, 4 lanes each
constexpr int RECG = 24;               // granules per MB record

// One unit's MB row in LDS.
struct alignas(16) UnitLds {
    uint32_t y[16][12];       // luma rows 0..15; MB x in slot s = x % 3: dwords 4s .. 4s+3
    uint32_t c[2][8][6];      // chroma plane, rows 0..7; slot s = dwords 2s, 2s+1
    uint32_t top[24];         // MB (x, y-1): luma rows -4..-1 [4][4], chroma [plane][rows -2, -1][2]
};
static_assert(sizeof(UnitLds) == 1248, "UnitLds layout");

typedef uint32_t v4u __attribute__((ext_vector_type(4)));   // native vectors: registers, not stack
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

DEV uint64_t ldcc64(const uint64_t* p) { return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DEV void stcc64(uint64_t* p, uint64_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// Record granule g -> dword of UnitLds::top.  0..11 luma rows -4..-1 dwords 0..2
// (3 per row), 12..15 chroma [plane][row] dword 0, 16..19 luma rows dword 3,
// 20..23 chroma [plane][row] dword 1.
DEV int top_index(int g)
{
    if (g < 12) return (g / 3) * 4 + g % 3;
    if (g < 16) return 16 + (g - 12) * 2;
    if (g < 20) return (g - 16) * 4 + 3;
    return 16 + (g - 20) * 2 + 1;
}

// {byte j, byte j + 2} of one dword as an s16x2 (the column pair (j, j+2)).
DEV s2 unpack_cols(uint32_t w, int j) { return as_s2(__builtin_amdgcn_perm(w, w, 0x0C000C00u | ((uint32_t)(j + 2) << 16) | (uint32_t)j)); }
// Column pairs (0, 2) and (1, 3) back into one dword.
DEV uint32_t pack_cols(s2 c0, s2 c1) { return __builtin_amdgcn_perm(as_w(c1), as_w(c0), 0x06020400u); }
DEV s2 bs_pair(uint32_t w, int slo, int shi) { return (s2){(short)((w >> (8 * slo)) & 255), (short)((w >> (8 * shi)) & 255)}; }

}  // namespace

// hb: records [pic][row & 1][W][RECG] granules {dword, tag}; sync[0]: ticket counter;
// epoch < 2^20 (the host restarts from zeroed records before it wraps).
extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_deblock2(h264r_batch b, const DbInfo* __restrict__ dbinfo, uint64_t* hb,
                                                            int* sync, int* err, uint32_t epoch, int2 rows)
{
    __shared__ UnitLds S[UNITS];
    const int lane = threadIdx.x, u = lane >> 2, q = lane & 3;
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int W = g.wmb, R0 = rows.x, R1 = rows.y;
    const int ngroups = (b.num_pics + UNITS - 1) / UNITS;
    int tk = 0;
    if (lane == 0) tk = atomicAdd(&sync[0], 1);
    const int ticket = __builtin_amdgcn_readfirstlane(tk);
    const int ry = ticket / ngroups, grp = ticket - ry * ngroups;
    const int y = R0 + ry;
    const int pic_raw = grp * UNITS + u;
    const bool active = pic_raw < b.num_pics;
    const int pic = active ? pic_raw : b.num_pics - 1;
    const bool above = y > R0, last_row = y == R1 - 1;
    // records live in two slots per picture (rows alternate); the tag names launch and row
    const uint64_t tag = (uint64_t)((epoch << 12) | ((uint32_t)ry & 0xFFFu)) << 32;
    const uint64_t tag_in = (uint64_t)((epoch << 12) | ((uint32_t)(ry - 1) & 0xFFFu)) << 32;

    UnitLds& U = S[u];
    const size_t Wl = (size_t)g.W, Wc = (size_t)g.Wc;
    uint8_t* Y = b.out_y + (size_t)pic * g.ysz + (size_t)(y * 16) * Wl;               // MB row y
    uint8_t* Cb = b.out_u + (size_t)pic * g.csz + (size_t)(y * 8) * Wc;
    uint8_t* Cr = b.out_v + (size_t)pic * g.csz + (size_t)(y * 8) * Wc;
    const int p = q >> 1;                                                               // my chroma plane
    uint8_t* Cp = p ? Cr : Cb;
    const v4u* info_row = reinterpret_cast<const v4u*>(dbinfo + (size_t)pic * g.nmb + (size_t)y * W);
    uint64_t* rec_out = hb + ((size_t)pic * 2 + (ry & 1)) * W * RECG;
    const uint64_t* rec_in = hb + ((size_t)pic * 2 + ((ry + 1) & 1)) * W * RECG;

    // ---- window fetch: MBs m, m+1 as 32-byte luma / 16-byte chroma row pieces
    v4u wl[8], wc[4];
    auto fetch = [&](int m) {
        const int xa = min(m + (q & 1), W - 1);
#pragma unroll
        for (int i = 0; i < 8; ++i) wl[i] = *reinterpret_cast<const v4u*>(Y + (size_t)(2 * i + (q >> 1)) * Wl + xa * 16);
        if (m + 1 < W) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int pr = 4 * i + q;                                               // plane * 8 + row
                wc[i] = *reinterpret_cast<const v4u*>((pr >> 3 ? Cr : Cb) + (size_t)(pr & 7) * Wc + m * 8);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int pr = 4 * i + q;
                const v2u v = *reinterpret_cast<const v2u*>((pr >> 3 ? Cr : Cb) + (size_t)(pr & 7) * Wc + m * 8);
                wc[i] = (v4u){v.x, v.y, 0u, 0u};
            }
        }
    };
    auto fill = [&](int m) {                                                            // registers -> ring slots
        const int sa = m % 3, sb = (m + 1) % 3, s = (q & 1) ? sb : sa;
#pragma unroll
        for (int i = 0; i < 8; ++i) *reinterpret_cast<v4u*>(&U.y[2 * i + (q >> 1)][4 * s]) = wl[i];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int pr = 4 * i + q;
            *reinterpret_cast<v2u*>(&U.c[pr >> 3][pr & 7][2 * sa]) = wc[i].xy;
            *reinterpret_cast<v2u*>(&U.c[pr >> 3][pr & 7][2 * sb]) = wc[i].zw;
        }
    };
    // MBs [m0, m1) are final: my luma rows 4q..4q+3 and chroma rows 4(q&1)..+3 of plane p
    auto store_mbs = [&](int m0, int m1) {
        if (!active) return;
        for (int m = m0; m < m1; ++m) {
            const int s = m % 3;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = 4 * q + i;
                if (r <= 12 || last_row)
                    *reinterpret_cast<v4u*>(Y + (size_t)r * Wl + m * 16) = *reinterpret_cast<const v4u*>(&U.y[r][4 * s]);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = 4 * (q & 1) + i;
                if (r <= 6 || last_row)
                    *reinterpret_cast<v2u*>(Cp + (size_t)r * Wc + m * 8) = *reinterpret_cast<const v2u*>(&U.c[p][r][2 * s]);
            }
        }
    };
    // the 8 granules of MB m that wait for MB m+1's vertical edges (luma dword 3, chroma dword 1)
    auto publish_b = [&](int m) {
        if (last_row || !active) return;
        const int s = m % 3;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int k = 2 * q + i;
            const uint32_t v = k < 4 ? U.y[12 + k][4 * s + 3] : U.c[(k - 4) >> 1][6 + ((k - 4) & 1)][2 * s + 1];
            stcc64(rec_out + (size_t)m * RECG + 16 + k, tag | v);
        }
    };

    uint32_t inf[20], ninf[20];
    auto load_info = [&](int x, uint32_t (&in)[20]) {
        const int xs = min(x, W - 1);
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const v4u v = info_row[(size_t)xs * 5 + k];
            in[4 * k] = v.x; in[4 * k + 1] = v.y; in[4 * k + 2] = v.z; in[4 * k + 3] = v.w;
        }
    };

    bool ok = true;
    fetch(0);
    fill(0);
    load_info(0, inf);
    __syncthreads();
    for (int x = 0; x < W; ++x) {
        const int sc = x % 3, sl = (x + 2) % 3;
        if (!(x & 1) && x + 2 < W) fetch(x + 2);                                        // next window
        if (x + 1 < W) load_info(x + 1, ninf);
        uint64_t rin[6];
        if (above) {
#pragma unroll
            for (int i = 0; i < 6; ++i) rin[i] = ldcc64(rec_in + (size_t)x * RECG + 6 * q + i);
        }

        // edge words of my chroma plane (par[3 + 3p ..], selected without indexing by p)
        const uint32_t cpar[3] = {p ? inf[14] : inf[11], p ? inf[15] : inf[12], p ? inf[16] : inf[13]};

        // ================= vertical edges of MB x (deblock.cc:488-504)
        {
            // luma rows (4q + i, 4q + i + 2): bS of V edge e, segment q = byte 4e + q
            EdgeP ev[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) ev[e] = edge_params(inf[8 + (e == 0 ? 0 : 2)], bs_pair(inf[e], q, q));
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int ra = 4 * q + i, rb = ra + 2;
                uint32_t la = U.y[ra][4 * sl + 3], lb = U.y[rb][4 * sl + 3];
                const v4u A = *reinterpret_cast<const v4u*>(&U.y[ra][4 * sc]);
                const v4u B = *reinterpret_cast<const v4u*>(&U.y[rb][4 * sc]);
                uint32_t a[4] = {A.x, A.y, A.z, A.w}, bb[4] = {B.x, B.y, B.z, B.w};
                s2 c[20];
#pragma unroll
                for (int k = 0; k < 4; ++k) c[k] = unpack2(la, lb, k);
#pragma unroll
                for (int k = 4; k < 20; ++k) c[k] = unpack2(a[(k >> 2) - 1], bb[(k >> 2) - 1], k & 3);
                filter2<true, false>(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], ev[0]);
#pragma unroll
                for (int e = 1; e < 4; ++e)
                    filter2<false, false>(c[4 * e], c[4 * e + 1], c[4 * e + 2], c[4 * e + 3], c[4 * e + 4], c[4 * e + 5],
                                          c[4 * e + 6], c[4 * e + 7], ev[e]);
                pack4(c[0], c[1], c[2], c[3], la, lb);
#pragma unroll
                for (int d = 0; d < 4; ++d) pack4(c[4 + 4 * d], c[5 + 4 * d], c[6 + 4 * d], c[7 + 4 * d], a[d], bb[d]);
                U.y[ra][4 * sl + 3] = la;
                U.y[rb][4 * sl + 3] = lb;
                *reinterpret_cast<v4u*>(&U.y[ra][4 * sc]) = (v4u){a[0], a[1], a[2], a[3]};
                *reinterpret_cast<v4u*>(&U.y[rb][4 * sc]) = (v4u){bb[0], bb[1], bb[2], bb[3]};
            }
            // chroma plane p rows (4(q&1) + i, +2); chroma edge 0 = luma edge 0, edge 1
            // (col 4) = luma edge 2; row j takes the bS of luma row 2j: segment j / 2
            // (deblock.cc:430-433, 460)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int ra = 4 * (q & 1) + i, rb = ra + 2;
                EdgeP ec[2];
#pragma unroll
                for (int e = 0; e < 2; ++e)
                    ec[e] = edge_params(cpar[e == 0 ? 0 : 2], bs_pair(inf[2 * e], ra >> 1, rb >> 1));
                uint32_t la = U.c[p][ra][2 * sl + 1], lb = U.c[p][rb][2 * sl + 1];
                const v2u A = *reinterpret_cast<const v2u*>(&U.c[p][ra][2 * sc]);
                const v2u B = *reinterpret_cast<const v2u*>(&U.c[p][rb][2 * sc]);
                uint32_t a[2] = {A.x, A.y}, bb[2] = {B.x, B.y};
                s2 c[12];
#pragma unroll
                for (int k = 0; k < 4; ++k) c[k] = unpack2(la, lb, k);
#pragma unroll
                for (int k = 4; k < 12; ++k) c[k] = unpack2(a[(k >> 2) - 1], bb[(k >> 2) - 1], k & 3);
                filter2<true, true>(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], ec[0]);
                filter2<false, true>(c[4], c[5], c[6], c[7], c[8], c[9], c[10], c[11], ec[1]);
                pack4(c[0], c[1], c[2], c[3], la, lb);
                pack4(c[4], c[5], c[6], c[7], a[0], bb[0]);
                pack4(c[8], c[9], c[10], c[11], a[1], bb[1]);
                U.c[p][ra][2 * sl + 1] = la;
                U.c[p][rb][2 * sl + 1] = lb;
                *reinterpret_cast<v2u*>(&U.c[p][ra][2 * sc]) = (v2u){a[0], a[1]};
                *reinterpret_cast<v2u*>(&U.c[p][rb][2 * sc]) = (v2u){bb[0], bb[1]};
            }
        }

        // ================= the record of MB (x, y-1) from the row above: wait for this launch
        if (above) {
            unsigned spins = 0;
            for (;;) {
                bool ready = true;
#pragma unroll
                for (int i = 0; i < 6; ++i) ready &= (rin[i] & 0xFFFFFFFF00000000ull) == tag_in;
                if (__all(ready || !active)) break;
                __builtin_amdgcn_s_sleep(1);
#pragma unroll
                for (int i = 0; i < 6; ++i) rin[i] = ldcc64(rec_in + (size_t)x * RECG + 6 * q + i);
                if (++spins > SPIN2) {
                    if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = false;
                    break;
                }
            }
            if (!ok) break;
#pragma unroll
            for (int i = 0; i < 6; ++i) U.top[top_index(6 * q + i)] = (uint32_t)rin[i];
        }
        // a band that starts below row 0 must not be filtered across its top edge (idc 1, or a
        // slice edge with idc 2): its top-edge strengths (bs[16..19] = info dword 4) are 0
        if (y == R0 && R0 > 0 && active && inf[4] != 0)
            __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();

        // MB x-1 is final for the row below now (its right columns after V(x))
        if (x >= 1) publish_b(x - 1);

        // ================= horizontal edges of MB x (deblock.cc:506-535)
        {
            // luma columns 4q .. 4q+3 (dword q), rows -4..15, pairs (4q + j, 4q + j + 2)
            uint32_t w[20];
#pragma unroll
            for (int r = 0; r < 4; ++r) w[r] = U.top[r * 4 + q];
#pragma unroll
            for (int r = 0; r < 16; ++r) w[4 + r] = U.y[r][4 * sc + q];
            EdgeP eh[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) eh[e] = edge_params(inf[8 + (e == 0 ? 1 : 2)], bs_pair(inf[4 + e], q, q));
            s2 c[2][20];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int r = 0; r < 20; ++r) c[j][r] = unpack_cols(w[r], j);
                filter2<true, false>(c[j][0], c[j][1], c[j][2], c[j][3], c[j][4], c[j][5], c[j][6], c[j][7], eh[0]);
#pragma unroll
                for (int e = 1; e < 4; ++e)
                    filter2<false, false>(c[j][4 * e], c[j][4 * e + 1], c[j][4 * e + 2], c[j][4 * e + 3], c[j][4 * e + 4],
                                          c[j][4 * e + 5], c[j][4 * e + 6], c[j][4 * e + 7], eh[e]);
            }
#pragma unroll
            for (int r = 1; r < 4; ++r) U.top[r * 4 + q] = pack_cols(c[0][r], c[1][r]);
#pragma unroll
            for (int r = 0; r < 16; ++r) U.y[r][4 * sc + q] = pack_cols(c[0][4 + r], c[1][4 + r]);
        }
        {
            // chroma plane p, columns 4(q&1) .. +3 (dword q&1), rows -2..7; the halves of a
            // pair sit in segments 2(q&1) and 2(q&1)+1 of luma H edge 0 / 2
            const int d = q & 1;
            uint32_t w[10];
#pragma unroll
            for (int r = 0; r < 2; ++r) w[r] = U.top[16 + p * 4 + r * 2 + d];
#pragma unroll
            for (int r = 0; r < 8; ++r) w[2 + r] = U.c[p][r][2 * sc + d];
            EdgeP eh[2];
#pragma unroll
            for (int e = 0; e < 2; ++e)
                eh[e] = edge_params(cpar[e == 0 ? 1 : 2], bs_pair(inf[4 + 2 * e], 2 * d, 2 * d + 1));
            s2 c[2][10];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int r = 0; r < 10; ++r) c[j][r] = unpack_cols(w[r], j);
                s2 d0 = c[j][0], d1 = c[j][9];
                filter2<true, true>(d0, d0, c[j][0], c[j][1], c[j][2], c[j][3], d1, d1, eh[0]);
                filter2<false, true>(d0, d0, c[j][4], c[j][5], c[j][6], c[j][7], d1, d1, eh[1]);
            }
            U.top[16 + p * 4 + 2 + d] = pack_cols(c[0][1], c[1][1]);
#pragma unroll
            for (int r = 0; r < 8; ++r) U.c[p][r][2 * sc + d] = pack_cols(c[0][2 + r], c[1][2 + r]);
        }
        __syncthreads();

        // ================= publish / store what is final now
        if (!last_row && active) {
            // the 16 granules of MB x that MB x+1 cannot change
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int k = 4 * q + i;
                const uint32_t v = k < 12 ? U.y[12 + k / 3][4 * sc + k % 3] : U.c[(k - 12) >> 1][6 + ((k - 12) & 1)][2 * sc];
                stcc64(rec_out + (size_t)x * RECG + k, tag | v);
            }
        }
        if (above && active) {
            // rows 13..15 of MB (x, y-1) (lanes 0..2), chroma row 7 of both planes (lane 3)
            if (q < 3) {
                *reinterpret_cast<v4u*>(Y - (size_t)(3 - q) * Wl + x * 16) = *reinterpret_cast<const v4u*>(&U.top[(1 + q) * 4]);
            } else {
                *reinterpret_cast<v2u*>(Cb - Wc + x * 8) = *reinterpret_cast<const v2u*>(&U.top[16 + 2]);
                *reinterpret_cast<v2u*>(Cr - Wc + x * 8) = *reinterpret_cast<const v2u*>(&U.top[16 + 4 + 2]);
            }
        }
        if ((x & 1) && x + 1 < W) {
            // window switch: MBs x-2, x-1 are final and leave the ring; x+1, x+2 come in
            store_mbs(max(x - 2, 0), x);
            __syncthreads();                         // every lane has read the slots fill() reuses
            fill(x + 1);
        }
        if (x + 1 < W) {
#pragma unroll
            for (int k = 0; k < 20; ++k) inf[k] = ninf[k];
        }
        __syncthreads();
    }
    if (ok) {
        // the row end: the MBs the last window switch left in the ring (three for even W,
        // two for odd W), and the last MB's late granules
        store_mbs(max(W - ((W & 1) ? 2 : 3), 0), W);
        publish_b(W - 1);
    } else if (!last_row) {                          // release the row below (the error is flagged)
        for (int x = 0; x < W; ++x)
            for (int k = q; k < RECG; k += 4) stcc64(rec_out + (size_t)x * RECG + k, tag);
    }
}
