// k_deblock.hip -- the in-loop deblocking filter of every picture of a batch.
//
// The reference filters MB by MB in raster order, vertical edges then
// horizontal edges (Deblock::deblock_pic, deblock.cc:537-552), and the result
// is order-dependent: MB (x,y)'s top edge reads samples that MB (x+1,y-1)'s
// left edge wrote, so MB (x,y) may start only once (x+1,y-1) is done -- a
// wavefront with a 2-MB lag per row.
//
// Work unit: one 64-lane wave owns a PAIR of MB rows (2p, 2p+1) of one
// picture.  Lanes 0..31 walk row 2p ("half A"), lanes 32..63 walk row 2p+1
// ("half B") two MBs behind, so every filter instruction works on two MBs
// and all 64 lanes are busy (per half: lanes 0..15 luma lines, 16..31 chroma
// lines).  Inside the pair, half A hands its bottom rows to half B through an
// LDS ring; between pairs, half B publishes each MB's final-for-it bottom rows
// as one self-validating record: 32 naturally aligned 8-byte granules {data
// dword, launch epoch}, written by one write-through (`sc1`) store instruction.
// The pair below reads the record with `sc1` loads and re-polls until every
// granule carries this launch's epoch (MI355X_MICROARCH.md, R2 granule
// hand-off): no progress counter, no `s_waitcnt vmcnt(0)` on the producer's
// path.  Pairs are taken as tickets from an atomic counter in
// pair-major order, so a wave only ever waits on a ticket taken earlier by a
// running wave: no deadlock under any dispatch order or residency; every spin
// is bounded and flags the error word.
//
// Sample ownership: each MB row writes its rows 0..12 (chroma 0..4) and the
// rows 13..15 (chroma 5..7) of the row above after filtering its top edge;
// only the picture's last row writes its own bottom rows.  A sample is stored
// once, when final, by exactly one wave.
#include "mb_deblock.h"

using namespace h264r;

namespace {

constexpr int DRING = 4;                    // row A -> row B ring depth (lag is 2)
constexpr unsigned SPIN_LIMIT = 1u << 22;   // ~0.3 s of polling, then flag an error

struct alignas(16) PairLds {
    DbLds t[2];                   // per half
    RingEntry ring[2][DRING];     // per half: bottom rows of the last MBs
};

DEV uint32_t ld_cc(const uint32_t* p)       // coherent (L1-bypassing, sc1) load
{
    return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DEV uint64_t ld_cc64(const uint64_t* p)     // coherent (L1-bypassing, sc1) 8-byte load
{
    return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DEV void st_cc64(uint64_t* p, uint64_t v)   // write-through (sc1) 8-byte store
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

#ifdef H264R_TRACE
// Experimental timing trace (exp/ builds only): per ticket {start, first step,
// end, cycles spent polling} in s_memrealtime ticks (100 MHz).
__device__ unsigned long long h264r_db_trace[1 << 16][8];
#define TRACE(...) __VA_ARGS__
extern "C" void h264r_db_trace_copy(void* dst) { (void)hipMemcpyFromSymbol(dst, HIP_SYMBOL(h264r_db_trace), sizeof(h264r_db_trace)); }
#else
#define TRACE(...)
#endif

// hb: hand-off records [pic][pair][W][32] granules {RingEntry dword, epoch};
// sync[0]: ticket counter; epoch: this launch's tag (never 0: hb is zeroed when allocated).
#ifndef H264R_DB_WAVES
#define H264R_DB_WAVES 1                    // minimum waves per SIMD asked of the register allocator
#endif
extern "C" __global__ __launch_bounds__(64, H264R_DB_WAVES) void k_deblock(h264r_batch b, const DbInfo* __restrict__ dbinfo,
                                                          uint64_t* hb, int* sync, int* err, uint32_t epoch, int2 rows)
{
    __shared__ PairLds L;
    const int lane = threadIdx.x, h = lane >> 5, hl = lane & 31;
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    // rows [R0, H): the MB rows decoded by this launch (a slice-aligned band, h264r_decode_batch_rows)
    const int W = g.wmb, R0 = rows.x, H = rows.y, npairs = (H - R0 + 1) >> 1;

    int tk = 0;
    if (lane == 0) tk = atomicAdd(&sync[0], 1);
    const int ticket = __builtin_amdgcn_readfirstlane(tk);
    TRACE(unsigned long long tr_start = __builtin_amdgcn_s_memrealtime();)
    const int rp = ticket / b.num_pics, pic = ticket % b.num_pics;
    const int r = R0 + 2 * rp + h;                         // this half's MB row
    const bool hasB = R0 + 2 * rp + 1 < H;
    const bool half_on = r < H;
    const bool last_row = r == H - 1;
    const bool feeds_ring = h == 0 && hasB;                // A -> B through LDS
    const bool feeds_hb = h == 1 && rp + 1 < npairs;       // B -> next pair through hb
    const uint64_t* hb_in = rp > 0 ? hb + ((size_t)pic * npairs + rp - 1) * W * 32 : nullptr;
    uint64_t* hb_out = hb + ((size_t)pic * npairs + rp) * W * 32;

    DbLds& S = L.t[h];
    uint32_t* Sw = reinterpret_cast<uint32_t*>(&S);        // tiles: Sw[p * TR * TP + (row + 4) * TP + dw]
    if (hl == 0) S.zero = 0;
    uint8_t* Y = b.out_y + (size_t)pic * g.ysz;
    uint8_t* Cp[2] = {b.out_u + (size_t)pic * g.csz, b.out_v + (size_t)pic * g.csz};
    const int Y0 = r * 16, Yc = r * 8;
    const uint32_t* info_row = reinterpret_cast<const uint32_t*>(dbinfo + (size_t)pic * g.nmb + (size_t)r * W);
    const uint64_t tag = (uint64_t)epoch << 32;
    const int steps = W + (hasB ? 2 : 0);

    // ---- per-lane roles (inside a half), computed once
    const int by0 = hl >> 2, bd0 = hl & 3;                 // luma body dwords hl and hl + 32
    const int cpl = hl >> 4, cy = (hl >> 1) & 7, cd = hl & 1;   // chroma body dword
    const int a_y0 = (4 + by0) * TP + 1 + bd0, a_y1 = a_y0 + 8 * TP;
    const int a_c = (1 + cpl) * TR * TP + (4 + cy) * TP + 1 + cd;
    const int a_top = hl < 16 ? (hl >> 2) * TP + 1 + (hl & 3)
                              : (1 + ((hl - 16) >> 3)) * TR * TP + (((hl - 16) >> 1) & 3) * TP + 1 + (hl & 1);
    // write-back slots: luma rows -3..15 x dwords 0..4 (95), chroma 2 x rows -3..7 x dwords 0..2 (66)
    constexpr int NWB = 6;
    int wb_word[NWB], wb_flags[NWB];                       // flags: 1 valid, 2 needs x > 0, 4 needs x == W-1, 8 chroma
    uint8_t* wb_ptr[NWB];
#pragma unroll
    for (int it = 0; it < NWB; ++it) {
        const int e = hl + 32 * it;
        int f = 0, word = 0;
        uint8_t* ptr = Y;
        if (e < 95) {
            const int row = e / 5 - 3, dw = e % 5;
            const bool v = row < 0 ? (r > R0 && dw >= 1) : (row <= 12 || last_row);
            f = (v ? 1 : 0) | (row >= 0 && dw == 0 ? 2 : 0) | (row >= 0 && dw == 4 ? 4 : 0);
            word = (row + 4) * TP + dw;
            ptr = Y + (ptrdiff_t)(Y0 + row) * g.W + 4 * (dw - 1);
        } else if (e < 161) {
            const int k = e - 95, pl = k / 33, k2 = k - pl * 33, row = k2 / 3 - 3, dw = k2 % 3;
            const bool v = row < 0 ? (r > R0 && dw >= 1) : (row <= 4 || last_row);
            f = (v ? 1 : 0) | (row >= 0 && dw == 0 ? 2 : 0) | (row >= 0 && dw == 2 ? 4 : 0) | 8;
            word = (1 + pl) * TR * TP + (row + 4) * TP + dw;
            ptr = Cp[pl] + (ptrdiff_t)(Yc + row) * g.Wc + 4 * (dw - 1);
        }
        wb_word[it] = word; wb_flags[it] = f; wb_ptr[it] = ptr;
    }
    // ring slots: luma rows 12..15 x dwords 0..4 (20), chroma 2 x rows 4..7 x dwords 0..2 (24)
    int rg_src[2], rg_dst[2], rg_kind[2];                  // kind: 0 entry x, 1 entry x-1 if x > 0, 2 entry x if last, 3 none
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const int e = hl + 32 * it;
        int src = 0, dst = 0, kind = 3;
        if (e < 20) {
            const int i = e / 5, dw = e % 5;
            src = (16 + i) * TP + dw;
            dst = i * 4 + (dw == 0 || dw == 4 ? 3 : dw - 1);
            kind = dw == 0 ? 1 : (dw == 4 ? 2 : 0);
        } else if (e < 44) {
            const int k = e - 20, pl = k / 12, k2 = k - pl * 12, i = k2 / 3, dw = k2 % 3;
            src = (1 + pl) * TR * TP + (8 + i) * TP + dw;
            dst = 16 + pl * 8 + i * 2 + (dw == 1 ? 0 : 1);
            kind = dw == 0 ? 1 : (dw == 2 ? 2 : 0);
        }
        rg_src[it] = src; rg_dst[it] = dst; rg_kind[it] = kind;
    }
    // carry slots: luma rows -4..15 (20), chroma 2 x rows -4..7 (24): dword 0 <- last dword
    int cy_src[2], cy_dst[2];
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const int e = hl + 32 * it;
        if (e < 20) { cy_dst[it] = e * TP; cy_src[it] = e * TP + 4; }
        else if (e < 44) {
            const int k = e - 20, pl = k / 12, row = k - pl * 12;
            cy_dst[it] = (1 + pl) * TR * TP + row * TP; cy_src[it] = cy_dst[it] + 2;
        } else { cy_dst[it] = -1; cy_src[it] = 0; }
    }

    uint32_t pf_y0 = 0, pf_y1 = 0, pf_c = 0, pf_i = 0;
    uint64_t pf_top = 0;
    bool ok = true;
    TRACE(unsigned long long tr_wait = 0; unsigned long long tph[4] = {0, 0, 0, 0}; unsigned long long tm = 0;)

    // Issue the loads of step t (this half's MB t - 2h): body, deblocking record
    // and, for half A below another pair, the hand-off record of the MB above.
    // The hand-off record is loaded first and unconditionally (lanes that do not need
    // it read their own output record): a conditional load merges into the
    // loop-carried register through a copy, and the copy's vmcnt(0) would retire the
    // whole prefetch at once instead of letting it overlap the filter work.
    auto prefetch = [&](int t) {
        const int x = t - 2 * h;
        const int xs = min(max(x, 0), W - 1);
        pf_top = ld_cc64(h == 0 && rp > 0 ? hb_in + (size_t)xs * 32 + hl : hb_out + hl);
        if (half_on && x >= 0 && x < W) {
            const uint8_t* yb = Y + (size_t)(Y0 + by0) * g.W + x * 16 + 4 * bd0;
            pf_y0 = *reinterpret_cast<const uint32_t*>(yb);
            pf_y1 = *reinterpret_cast<const uint32_t*>(yb + (size_t)8 * g.W);
            pf_c = *as_global(Cp[cpl] + (size_t)(Yc + cy) * g.Wc + x * 8 + 4 * cd);
            if (hl < DBINFO_DWORDS) pf_i = info_row[x * DBINFO_DWORDS + hl];
        }
    };

    prefetch(0);
    TRACE(const unsigned long long tr_first = __builtin_amdgcn_s_memrealtime();)
    for (int t = 0; t < steps; ++t) {
        const int x = t - 2 * h;
        const bool act = half_on && x >= 0 && x < W;

        // ---- the record of the MB above (half A below another pair): wait for this epoch
        if (rp > 0) {
            const bool need = act && h == 0;
            unsigned spins = 0;
            TRACE(unsigned long long tw0 = 0;)
            while (!__all(!need || (pf_top & 0xFFFFFFFF00000000ull) == tag)) {
                TRACE(if (!tw0) tw0 = __builtin_amdgcn_s_memrealtime();)
                __builtin_amdgcn_s_sleep(1);
                if (need) pf_top = ld_cc64(hb_in + (size_t)x * 32 + hl);
                if (++spins > SPIN_LIMIT) {
                    if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = false;
                    break;
                }
            }
            TRACE(if (tw0) tr_wait += __builtin_amdgcn_s_memrealtime() - tw0;)
            if (!ok) break;
        }
        TRACE(unsigned long long ta = __builtin_amdgcn_s_memtime();)
        // ---- assemble the tiles (an idle half scribbles on its own tiles only)
        Sw[a_y0] = pf_y0;
        Sw[a_y1] = pf_y1;
        Sw[a_c] = pf_c;
        if (hl < DBINFO_DWORDS) S.info[hl] = pf_i;
        // a band that starts below row 0 must not be filtered across its top edge (idc 1 or
        // a slice edge with idc 2): its top-edge strengths (bs[16..19] = info dword 4) are 0
        if (r == R0 && R0 > 0 && act && hl == 4 && pf_i != 0)
            __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (r > R0) Sw[a_top] = h == 0 ? (uint32_t)pf_top : reinterpret_cast<const uint32_t*>(&L.ring[0][x & (DRING - 1)])[hl];
        TRACE(asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); tph[0] += __builtin_amdgcn_s_memtime() - ta;)
        if (t + 1 < steps) prefetch(t + 1);
        wave_sync();
        TRACE(tm = __builtin_amdgcn_s_memtime();)
        filter_mb(S, hl);
        TRACE(asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); { unsigned long long t2 = __builtin_amdgcn_s_memtime(); tph[1] += t2 - tm; tm = t2; })

        // ---- write back what is final (see the header comment)
        const bool xl = x > 0, xr = x == W - 1;
#pragma unroll
        for (int it = 0; it < NWB; ++it) {
            const int f = wb_flags[it];
            const bool v = act && (f & 1) && (xl || !(f & 2)) && (xr || !(f & 4));
            if (v) *reinterpret_cast<uint32_t*>(wb_ptr[it] + x * ((f & 8) ? 8 : 16)) = Sw[wb_word[it]];
        }
        // ---- bottom rows of MB x (cols 0..11) and MB x-1 (cols 12..15) into this half's ring
        if (act && (feeds_ring || feeds_hb)) {
            uint32_t* ring = reinterpret_cast<uint32_t*>(L.ring[h]);
#pragma unroll
            for (int it = 0; it < 2; ++it) {
                const int k = rg_kind[it];
                const int ent = k == 1 ? (x + DRING - 1) & (DRING - 1) : x & (DRING - 1);
                if (k == 0 || (k == 1 && xl) || (k == 2 && xr)) ring[ent * 32 + rg_dst[it]] = Sw[rg_src[it]];
            }
        }
        wave_sync();
        TRACE({ unsigned long long t2 = __builtin_amdgcn_s_memtime(); tph[2] += t2 - tm; tm = t2; })
        // ---- half B: completed records (MB x-1, and MB x at the row end) to the hand-off buffer
        if (act && feeds_hb) {
            const uint32_t* ring = reinterpret_cast<const uint32_t*>(L.ring[1]);
            if (xl) st_cc64(hb_out + (size_t)(x - 1) * 32 + hl, tag | ring[((x + DRING - 1) & (DRING - 1)) * 32 + hl]);
            if (xr) st_cc64(hb_out + (size_t)x * 32 + hl, tag | ring[(x & (DRING - 1)) * 32 + hl]);
        }
        // ---- carry the right 4 columns into the left strip of the next tile
#pragma unroll
        for (int it = 0; it < 2; ++it)
            if (cy_dst[it] >= 0) Sw[cy_dst[it]] = Sw[cy_src[it]];
        wave_sync();
        TRACE({ unsigned long long t2 = __builtin_amdgcn_s_memtime(); tph[3] += t2 - tm; })
    }
    if (!ok && feeds_hb)                                   // release the pair below (the error is flagged)
        for (int x = 0; x < W; ++x) st_cc64(hb_out + (size_t)x * 32 + hl, tag);
    TRACE(if (lane == 0 && ticket < (1 << 16)) {
        h264r_db_trace[ticket][0] = tr_start; h264r_db_trace[ticket][1] = tr_first;
        h264r_db_trace[ticket][2] = __builtin_amdgcn_s_memrealtime(); h264r_db_trace[ticket][3] = tr_wait;
        for (int i = 0; i < 4; ++i) h264r_db_trace[ticket][4 + i] = tph[i]; })
}
