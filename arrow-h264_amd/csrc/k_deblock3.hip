// k_deblock3.hip -- the row walk of k_deblock2 with EIGHT lanes per (picture, MB row) unit
// and eight pictures per wave (k_deblock2: four lanes, sixteen pictures).
//
// Same schedule, hand-off records and sample ownership as k_deblock2 (k_deblock2.hip,
// whose header explains them); what changes is the lane split of one unit's work:
//
//   vertical edges   lane q filters the luma line pair (4(q>>1) + (q&1), +2) and the
//                    chroma pair (4((q&3)>>1) + (q&1), +2) of plane q>>2
//   horizontal edges lane q filters the luma column pair (4(q>>1) + (q&1), +2) and the
//                    chroma column pair (4((q>>1)&1) + (q&1), +2) of plane q>>2; the two
//                    lanes of a dword merge their bytes through a lane swap
//
// so a lane carries half of k_deblock2's filter state (fewer VGPRs) and a wave half of its
// LDS (8 x 1264 B): more waves per SIMD, each step half as long.  The hand-off records keep
// k_deblock2's layout: lanes 2c and 2c+1 poll consumer c's six granules.
#include <type_traits>

#include "mb_deblock.h"
#include "mb_deblock2.h"

using namespace h264r;

namespace {

#ifndef H264R_DB3_WAVES
#define H264R_DB3_WAVES 3              // waves per SIMD asked of the register allocator
#endif
constexpr int UNITS3 = 8;              // (picture, MB row) units per wave, 8 lanes each
constexpr int RECG = 24;               // granules per MB record: [consumer lane c 0..3][i 0..5]
constexpr int AUX_SC1 = 16;            // buffer-op cache policy: sc1 (write-through store, L2-served load)

struct alignas(16) UnitLds3 {
    uint32_t y[16][12];       // luma rows 0..15; MB x in slot s = x % 3: dwords 4s .. 4s+3
    uint32_t c[2][8][6];      // chroma plane, rows 0..7; slot s = dwords 2s, 2s+1
    uint32_t info[20];        // DbInfo of the MB being filtered
    uint32_t pad[8];
};
static_assert(sizeof(UnitLds3) == 1264, "UnitLds3 layout");

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

DEV s2 unpack_cols(uint32_t w, int j) { return as_s2(__builtin_amdgcn_perm(w, w, 0x0C000C00u | ((uint32_t)(j + 2) << 16) | (uint32_t)j)); }
// bytes j, j+2 of a dword from the halves of one column pair (the other bytes 0)
DEV uint32_t place_cols(s2 c, int j) { return (((uint32_t)(uint8_t)c.x) | ((uint32_t)(uint8_t)c.y << 16)) << (8 * j); }
DEV s2 bs_pair(uint32_t w, int slo, int shi) { return (s2){(short)((w >> (8 * slo)) & 255), (short)((w >> (8 * shi)) & 255)}; }

}  // namespace

extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(H264R_DB3_WAVES))) void k_deblock3(
    h264r_batch b, const DbInfo* __restrict__ dbinfo, uint64_t* hb, int* sync, int* err, uint32_t epoch, int2 rows, int nx,
    const uint8_t* __restrict__ recon)
{
    __shared__ UnitLds3 S[UNITS3];
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int W = g.wmb, R0 = rows.x, R1 = rows.y;
    const int ngroups = (b.num_pics + UNITS3 - 1) / UNITS3;
    unsigned xcc_reg = 0;
    if (nx > 1) asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_reg));
    const int xcc = (int)(xcc_reg & 15u) % nx;
    const int ngx = (ngroups - xcc + nx - 1) / nx;           // groups xcc, xcc + nx, ...
    int* counter = &sync[xcc];
    const bool local = nx > 1;
    const int items = ngx * (R1 - R0);
    for (;;) {
    __syncthreads();
    int tk = 0;
    if (threadIdx.x == 0) tk = atomicAdd(counter, 1);
    const int ticket = __builtin_amdgcn_readfirstlane(tk);
    if (ticket >= items) {
        xcd_drain_check(sync, sync + 8, nx, [&](int k) { return (ngroups - k + nx - 1) / nx * (R1 - R0); }, err);
        return;
    }
    const int ry = ticket / ngx, grp = (ticket - ry * ngx) * nx + xcc;
    int lane = threadIdx.x;
    asm volatile("" : "+v"(lane));
    const int u = lane >> 3;
    int q = lane & 7;
    int c4 = q >> 1, j = q & 1;                                // consumer lane of k_deblock2, column pair
    int p = q >> 2;                                            // my chroma plane
    const int y = R0 + ry;
    const int pic_raw = grp * UNITS3 + u;
    const bool active = pic_raw < b.num_pics;
    const int pic = active ? pic_raw : b.num_pics - 1;
    const bool above = y > R0, last_row = y == R1 - 1;
    const uint32_t tag32 = (epoch << 12) | ((uint32_t)ry & 0xFFFu);
    const uint64_t tag_in = (uint64_t)((epoch << 12) | ((uint32_t)(ry - 1) & 0xFFFu)) << 32;

    UnitLds3& U = S[u];
    const size_t Wl = (size_t)g.W, Wc = (size_t)g.Wc;
    uint8_t* Y = b.out_y + (size_t)pic * g.ysz + (size_t)(y * 16) * Wl;
    uint8_t* Cb = b.out_u + (size_t)pic * g.csz + (size_t)(y * 8) * Wc;
    uint8_t* Cr = b.out_v + (size_t)pic * g.csz + (size_t)(y * 8) * Wc;
    uint8_t* Cp = p ? Cr : Cb;
    const v4u* info_row = reinterpret_cast<const v4u*>(dbinfo + (size_t)pic * g.nmb + (size_t)y * W);
    const uint32_t hb_bytes = (uint32_t)b.num_pics * 2u * (uint32_t)W * RECG * 8u;
    const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc(hb, 0, hb_bytes, 0x00020000);
    const uint32_t rec_out = (uint32_t)(((size_t)pic * 2 + (ry & 1)) * W * RECG * 8);
    const uint32_t rec_in = (uint32_t)(((size_t)pic * 2 + ((ry + 1) & 1)) * W * RECG * 8);
    // record pair layout of k_deblock2 (three 64-byte blocks per MB)
    auto pair_off = [&](uint32_t base, int m, int c, int k) -> uint32_t {
        const int blk = c == 0 ? 0 : c == 2 ? 1 : c == 3 ? 2 : (k < 2 ? k : 2);
        const int slot = c == 0 || c == 2 ? k : c == 3 ? k + 1 : (k < 2 ? 3 : 0);
        return base + (uint32_t)(m * RECG) * 8u + (uint32_t)(blk * 4 + slot) * 16u;
    };
    auto load_pair = [&](int m, int k) -> v4u {
        return __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(hrs, pair_off(rec_in, m, c4, k), 0, AUX_SC1));
    };

    // ---- window fetch: MBs m, m+1 (768 contiguous bytes of the tiled reconstruction), six
    // 16-byte loads per lane: luma piece k = q + 8i (MB m + k / 16, row k % 16), chroma
    // chunk k = q + 8i (MB m + k / 8, plane (k / 4) & 1, rows 2 (k & 3), +1)
    const uint8_t* rrow = recon + ((size_t)pic * g.nmb + (size_t)y * W) * RECON_MB;
    v4u wl[4], wc[2];
    auto fetch = [&](int m) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = q + 8 * i;
            wl[i] = load_global<v4u>(rrow + (size_t)min(m + (k >> 4), W - 1) * RECON_MB + (k & 15) * 16);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int k = q + 8 * i;
            wc[i] = load_global<v4u>(rrow + (size_t)min(m + (k >> 3), W - 1) * RECON_MB + RECON_CB + (k & 7) * 16);
        }
    };
    auto fill = [&](int m) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = q + 8 * i, s = (m + (k >> 4)) % 3;
            *reinterpret_cast<v4u*>(&U.y[k & 15][4 * s]) = wl[i];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int k = q + 8 * i, s = (m + (k >> 3)) % 3, pl = (k >> 2) & 1, r = 2 * (k & 3);
            *reinterpret_cast<v2u*>(&U.c[pl][r][2 * s]) = wc[i].xy;
            *reinterpret_cast<v2u*>(&U.c[pl][r + 1][2 * s]) = wc[i].zw;
        }
    };
    auto consume_window = [&]() {
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(wl[i]));
#pragma unroll
        for (int i = 0; i < 2; ++i) asm volatile("" ::"v"(wc[i]));
    };
    const int ylast = last_row ? 15 : 12, clast = last_row ? 7 : 6;
    // final MBs m, m+1: piece k = q + 8i is row k / 2 of MB m + (k & 1) (two lanes make one
    // 32-byte row piece); chroma piece k: plane-row k / 2 of MB m + (k & 1)
    auto store_pair = [&](int m) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = q + 8 * i, r = min(k >> 1, ylast), mm = m + (k & 1);
            *reinterpret_cast<v4u*>(Y + (size_t)r * Wl + mm * 16) = *reinterpret_cast<const v4u*>(&U.y[r][4 * (mm % 3)]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = q + 8 * i, pr = k >> 1, r = min(pr & 7, clast), mm = m + (k & 1);
            uint8_t* dst = (pr >> 3 ? Cr : Cb) + (size_t)r * Wc + mm * 8;
            *reinterpret_cast<v2u*>(dst) = *reinterpret_cast<const v2u*>(&U.c[pr >> 3][r][2 * (mm % 3)]);
        }
    };
    auto store_one = [&](int m) {
        const int s = m % 3;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int r = min(2 * q + i, ylast);
            *reinterpret_cast<v4u*>(Y + (size_t)r * Wl + m * 16) = *reinterpret_cast<const v4u*>(&U.y[r][4 * s]);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int r = min(2 * (q & 3) + i, clast);
            *reinterpret_cast<v2u*>(Cp + (size_t)r * Wc + m * 8) = *reinterpret_cast<const v2u*>(&U.c[p][r][2 * s]);
        }
    };
    auto granule = [&](int m, int c, int i) -> uint32_t {
        const int s = m % 3;
        return i < 4 ? U.y[12 + i][4 * s + c] : U.c[c >> 1][2 + i][2 * s + (c & 1)];
    };
    auto publish_pair = [&](int m, int c, int k, uint32_t t) {
        const v4u v = {granule(m, c, 2 * k), t, granule(m, c, 2 * k + 1), t};
        const auto w = __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v);
        if (local) __builtin_amdgcn_raw_buffer_store_b128(w, hrs, pair_off(rec_out, m, c, k), 0, 0);
        else __builtin_amdgcn_raw_buffer_store_b128(w, hrs, pair_off(rec_out, m, c, k), 0, AUX_SC1);
    };
    // early pairs (final after H(x)): 8, lane q -> block q / 4 slot q % 4; late pairs (final
    // after V(x+1)): 4, lanes 0..3 -> block 2 slot q (lanes 4..7 repeat lanes 0..3's)
    const int lq = q & 3, jb = q >> 2;
    const int e_c = lq < 3 ? (jb ? 2 : 0) : 1, e_k = lq < 3 ? lq : jb;
    const int l_c = lq == 0 ? 1 : 3, l_k = lq == 0 ? 2 : lq - 1;
    // DbInfo of MB m: 5 pieces of 16 bytes, lane q < 5 one each
    v4u ninf;
    auto load_info = [&](int m) { ninf = info_row[(size_t)min(m, W - 1) * 5 + min(q, 4)]; };
    auto put_info = [&]() { if (q < 5) *reinterpret_cast<v4u*>(&U.info[4 * q]) = ninf; };

    bool ok = true;
    fetch(0);
    load_info(0);
    fill(0);
    put_info();
    __syncthreads();
    auto step = [&](const int x, auto odd_tag) {
        constexpr bool ODD = decltype(odd_tag)::value;
        // the lane role, opaque per step: what derives from it (addresses) is recomputed per
        // step, not kept live across the walk
        asm volatile("" : "+v"(q));
        c4 = q >> 1; j = q & 1; p = q >> 2;
        const int sc = x % 3, sl = (x + 2) % 3;
        // 1. the record of MB (x, y-1) (checked after the vertical edges)
        uint64_t rin[6];
        if (above) {
#pragma unroll
            for (int k = 0; k < 3; ++k) { const v4u v = load_pair(x, k); rin[2 * k] = v.x | (uint64_t)v.y << 32; rin[2 * k + 1] = v.z | (uint64_t)v.w << 32; }
        }
        load_info(x + 1);
        // DbInfo words read from LDS where they are used (held in registers across the step
        // they cost 20 VGPRs): [0..3] V bS, [4..7] H bS, [8..10] luma edge words, [11..16]
        // chroma (Cb: 11..13, Cr: 14..16)
        auto inf = [&](int k) -> uint32_t { return U.info[k]; };
        auto cpar = [&](int k) -> uint32_t { return U.info[11 + 3 * p + k]; };

        // 2. vertical edges of MB x (deblock.cc:488-504): one luma and one chroma line pair
        {
            // edge parameters made where each edge is filtered (all four live cost 20 VGPRs)
            auto ev = [&](int e) { return edge_params(inf(8 + (e == 0 ? 0 : 2)), bs_pair(inf(e), c4, c4)); };
            const int ra = 4 * c4 + j, rb = ra + 2;
            uint32_t la = U.y[ra][4 * sl + 3], lb = U.y[rb][4 * sl + 3];
            const v4u A = *reinterpret_cast<const v4u*>(&U.y[ra][4 * sc]);
            const v4u B = *reinterpret_cast<const v4u*>(&U.y[rb][4 * sc]);
            uint32_t a[4] = {A.x, A.y, A.z, A.w}, bb[4] = {B.x, B.y, B.z, B.w};
            s2 c[20];
#pragma unroll
            for (int k = 0; k < 4; ++k) c[k] = unpack2(la, lb, k);
#pragma unroll
            for (int k = 4; k < 20; ++k) c[k] = unpack2(a[(k >> 2) - 1], bb[(k >> 2) - 1], k & 3);
            filter2<true, false>(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], ev(0));
#pragma unroll
            for (int e = 1; e < 4; ++e)
                filter2<false, false>(c[4 * e], c[4 * e + 1], c[4 * e + 2], c[4 * e + 3], c[4 * e + 4], c[4 * e + 5],
                                      c[4 * e + 6], c[4 * e + 7], ev(e));
            pack4(c[0], c[1], c[2], c[3], la, lb);
#pragma unroll
            for (int k = 0; k < 4; ++k) pack4(c[4 + 4 * k], c[5 + 4 * k], c[6 + 4 * k], c[7 + 4 * k], a[k], bb[k]);
            U.y[ra][4 * sl + 3] = la;
            U.y[rb][4 * sl + 3] = lb;
            *reinterpret_cast<v4u*>(&U.y[ra][4 * sc]) = (v4u){a[0], a[1], a[2], a[3]};
            *reinterpret_cast<v4u*>(&U.y[rb][4 * sc]) = (v4u){bb[0], bb[1], bb[2], bb[3]};
        }
        {
            const int k2 = q & 3, ra = 4 * (k2 >> 1) + (k2 & 1), rb = ra + 2;
            EdgeP ec[2];
#pragma unroll
            for (int e = 0; e < 2; ++e)
                ec[e] = edge_params(cpar(e == 0 ? 0 : 2), bs_pair(inf(2 * e), ra >> 1, rb >> 1));
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
        // 3. the next window, behind the record loads in issue order
        if (!ODD) fetch(min(x + 2, W - 1));

        // 4. the record of MB (x, y-1) from the row above: wait for this launch
        if (above) {
            auto ready = [&]() {
                bool r = true;
#pragma unroll
                for (int i = 0; i < 6; ++i) r &= (rin[i] & 0xFFFFFFFF00000000ull) == tag_in;
                return __builtin_amdgcn_readfirstlane(__all(r || !active)) != 0;
            };
            if (!ready()) {
                WaitClock wck;
                do {
                    __builtin_amdgcn_s_sleep(1);
#pragma unroll
                    for (int k = 0; k < 3; ++k) { const v4u v = load_pair(x, k); rin[2 * k] = v.x | (uint64_t)v.y << 32; rin[2 * k + 1] = v.z | (uint64_t)v.w << 32; }
                    if (wait_give_up(err, wck)) {
                        ok = false;
                        consume_window();
                        return;
                    }
                } while (!ready());
            }
        }
        if (y == R0 && R0 > 0 && __builtin_amdgcn_readfirstlane(__any(active && inf(4) != 0)))
            __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        // the late pairs of MB x-1, final after V(x); tag 0 at x = 0 (never taken for ready)
        publish_pair(max(x - 1, 0), l_c, l_k, x ? tag32 : 0u);

        // 5. horizontal edges of MB x (deblock.cc:506-535): one luma and one chroma column
        // pair; the two lanes of a dword merge their bytes after the filters
        uint32_t wy[20], wcv[10];
        {
#pragma unroll
            for (int r = 0; r < 4; ++r) wy[r] = (uint32_t)rin[r];
#pragma unroll
            for (int r = 0; r < 16; ++r) wy[4 + r] = U.y[r][4 * sc + c4];
            auto eh = [&](int e) { return edge_params(inf(8 + (e == 0 ? 1 : 2)), bs_pair(inf(4 + e), c4, c4)); };
            s2 c[20];
#pragma unroll
            for (int r = 0; r < 20; ++r) c[r] = unpack_cols(wy[r], j);
            filter2<true, false>(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], eh(0));
#pragma unroll
            for (int e = 1; e < 4; ++e)
                filter2<false, false>(c[4 * e], c[4 * e + 1], c[4 * e + 2], c[4 * e + 3], c[4 * e + 4], c[4 * e + 5],
                                      c[4 * e + 6], c[4 * e + 7], eh(e));
#pragma unroll
            for (int r = 1; r < 20; ++r) {
                const uint32_t mine = place_cols(c[r], j);
                wy[r] = mine | (uint32_t)__shfl_xor((int)mine, 1);
            }
            if (j == 0) {
#pragma unroll
                for (int r = 0; r < 16; ++r) U.y[r][4 * sc + c4] = wy[4 + r];
            }
        }
        {
            const int d = c4 & 1;
#pragma unroll
            for (int r = 0; r < 2; ++r) wcv[r] = (uint32_t)rin[4 + r];
#pragma unroll
            for (int r = 0; r < 8; ++r) wcv[2 + r] = U.c[p][r][2 * sc + d];
            EdgeP eh[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) eh[e] = edge_params(cpar(e == 0 ? 1 : 2), bs_pair(inf(4 + 2 * e), 2 * d, 2 * d + 1));
            s2 c[10];
#pragma unroll
            for (int r = 0; r < 10; ++r) c[r] = unpack_cols(wcv[r], j);
            s2 d0 = c[0], d1 = c[9];
            filter2<true, true>(d0, d0, c[0], c[1], c[2], c[3], d1, d1, eh[0]);
            filter2<false, true>(d0, d0, c[4], c[5], c[6], c[7], d1, d1, eh[1]);
#pragma unroll
            for (int r = 1; r < 10; ++r) {
                const uint32_t mine = place_cols(c[r], j);
                wcv[r] = mine | (uint32_t)__shfl_xor((int)mine, 1);
            }
            if (j == 0) {
#pragma unroll
                for (int r = 0; r < 8; ++r) U.c[p][r][2 * sc + d] = wcv[2 + r];
            }
        }
        wave_sync();

        // 6. publish / store what is final now
        publish_pair(x, e_c, e_k, tag32);
        if (x == W - 1) publish_pair(x, l_c, l_k, tag32);
        if (above) {
            // rows 13..15 of MB (x, y-1): lane j = 0 of each dword; chroma row 7: lane j = 1
            if (j == 0) {
#pragma unroll
                for (int r = 1; r < 4; ++r) *reinterpret_cast<uint32_t*>(Y - (size_t)(4 - r) * Wl + x * 16 + 4 * c4) = wy[r];
            } else {
                *reinterpret_cast<uint32_t*>(Cp - Wc + x * 8 + 4 * (c4 & 1)) = wcv[1];
            }
        }
        __syncthreads();
        if (ODD) {
            if (x + 1 < W) {
                store_pair(max(x - 2, 0));
                __syncthreads();
                fill(x + 1);
            } else {
                consume_window();
            }
        }
        put_info();
        __syncthreads();
    };
    for (int x = 0;; x += 2) {
        step(x, std::false_type());
        if (!ok || x + 1 >= W) break;
        step(x + 1, std::true_type());
        if (!ok || x + 2 >= W) break;
    }
    if (ok) {
        const int m0 = max(W - ((W & 1) ? 2 : 3), 0);
        if (W - m0 == 3) { store_pair(m0); store_one(m0 + 2); }
        else if (W - m0 == 2) store_pair(m0);
        else store_one(m0);
    } else if (!last_row) {                          // release the row below (the error is flagged)
        for (int x = 0; x < W; ++x)
            for (int k = 0; k < 3; ++k) {
                const v4u v = {0u, tag32, 0u, tag32};
                const auto w = __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v);
                if (q < 4) {
                    if (local) __builtin_amdgcn_raw_buffer_store_b128(w, hrs, pair_off(rec_out, x, q, k), 0, 0);
                    else __builtin_amdgcn_raw_buffer_store_b128(w, hrs, pair_off(rec_out, x, q, k), 0, AUX_SC1);
                }
            }
    }
    }
}
