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
// ("half B") one MB behind, so every filter instruction works on two MBs
// and all 64 lanes are busy (per half: lanes 0..15 luma lines, 16..31 chroma
// lines).  One MB behind is the least lag the reference's order allows: MB
// (x, y)'s horizontal edges need (x+1, y-1)'s vertical edges only (they change
// columns 13..15 of (x, y-1)), so a step runs the vertical edges of both halves,
// then hands the bottom rows of the MB above to each half, then the horizontal
// edges.  Inside the pair, half A hands its bottom rows to half B through an
// LDS ring; between pairs, half B publishes each MB's final-for-it bottom rows
// as one self-validating record: 32 naturally aligned 8-byte granules {data
// dword, launch epoch}, written by one write-through (`sc1`) store instruction,
// as soon as the vertical edges of the MB to its right are done.
// The pair below reads the record with `sc1` loads and re-polls until every
// granule carries this launch's epoch (MI355X_MICROARCH.md, R2 granule
// hand-off): no progress counter, no `s_waitcnt vmcnt(0)` on the producer's
// path.  Pairs are taken as tickets from an atomic counter in
// pair-major order, so a wave only ever waits on a ticket taken earlier by a
// running wave: no deadlock under any dispatch order or residency; every spin
// is bounded and flags the error word.  A pair trails the pair above by two
// steps plus the hand-off (profiles/r02_deblock_lone_trace.txt).
//
// Sample ownership: each MB row writes its rows 0..12 (chroma 0..4) and the
// rows 13..15 (chroma 5..7) of the row above after filtering its top edge;
// only the picture's last row writes its own bottom rows.  A sample is stored
// once, when final, by exactly one wave.
#include "mb_deblock.h"

using namespace h264r;

namespace {

constexpr int DRING = 4;                    // row A -> row B ring depth (lag is 1)

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
// a hand-off record granule: plain (kept in the XCD's L2) when producer and consumer share
// the XCD (local), else write-through
DEV void st_rec(uint64_t* p, uint64_t v, bool local)
{
    if (local) *(__attribute__((address_space(1))) uint64_t*)p = v;
    else st_cc64(p, v);
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
// nx > 1: XCD-local hand-off, as in k_deblock2 -- every pair of a picture on one XCD
// (picture p on XCD p % nx, per-XCD ticket counters sync[0 .. nx-1], the XCD read from
// HW_REG_XCC_ID; waves take tickets until their XCD's run out) and the records as plain
// stores kept in that XCD's L2.  The host launches nx times the pairs of the largest XCD
// share, so each XCD's pairs all run at once whatever the round-robin start.
extern "C" __global__ __launch_bounds__(64, H264R_DB_WAVES) void k_deblock(h264r_batch b, const DbInfo* __restrict__ dbinfo,
                                                          uint64_t* hb, int* sync, int* err, uint32_t epoch, int2 rows,
                                                          int nx, uint8_t* recon)
{
    __shared__ PairLds L;
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    // rows [R0, H): the MB rows decoded by this launch (a slice-aligned band, h264r_decode_batch_rows)
    const int W = g.wmb, R0 = rows.x, H = rows.y, npairs = (H - R0 + 1) >> 1;
    unsigned xcc_reg = 0;
    if (nx > 1) asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_reg));
    const int xcc = (int)(xcc_reg & 15u) % nx;
    const int npx = (b.num_pics - xcc + nx - 1) / nx;          // pictures xcc, xcc + nx, ...
    const bool local = nx > 1;
    const int items = npx * npairs;
    for (;;) {
    __syncthreads();                                          // the previous item's LDS use is over
    int lane = threadIdx.x;
    asm volatile("" : "+v"(lane));                            // per item: no hoisted lane-derived state
    const int h = lane >> 5, hl = lane & 31;
    int tk = 0;
    if (lane == 0) tk = atomicAdd(&sync[xcc], 1);
    const int ticket = __builtin_amdgcn_readfirstlane(tk);
    if (ticket >= items) {
        xcd_drain_check(sync, sync + 8, nx, [&](int k) { return (b.num_pics - k + nx - 1) / nx * npairs; }, err);
        return;
    }
    TRACE(unsigned long long tr_start = __builtin_amdgcn_s_memrealtime();)
    const int rp = ticket / npx, pic = (ticket - rp * npx) * nx + xcc;
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
    const int steps = W + (hasB ? 1 : 0);

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
    uint64_t top = 0;
    bool ok = true;
    TRACE(unsigned long long tr_wait = 0; unsigned long long tph[4] = {0, 0, 0, 0}; unsigned long long tm = 0;)

    // The body loads of step t (this half's MB t - h): samples (the MB-tiled reconstruction,
    // device_common.h) and deblocking record.
    auto prefetch = [&](int t) {
        const int x = t - h;
        if (half_on && x >= 0 && x < W) {
            const uint8_t* mb = recon_mb(recon, g, pic, r * W + x);
            pf_y0 = load_global<uint32_t>(mb + by0 * 16 + 4 * bd0);
            pf_y1 = load_global<uint32_t>(mb + (by0 + 8) * 16 + 4 * bd0);
            pf_c = load_global<uint32_t>(mb + RECON_CB + cpl * 64 + cy * 8 + 4 * cd);
            if (hl < DBINFO_DWORDS) pf_i = info_row[x * DBINFO_DWORDS + hl];
        }
    };
    // The hand-off record of MB x above (half A below another pair), loaded first in a
    // step and unconditionally (lanes that do not need it read their own output
    // record): a conditional load merges into its register through a copy, whose
    // vmcnt(0) would retire the body prefetch with it.  The vertical edges cover it.
    auto load_top = [&](int x) {
        const int xs = min(max(x, 0), W - 1);
        top = ld_cc64(h == 0 && rp > 0 ? hb_in + (size_t)xs * 32 + hl : hb_out + hl);
    };
    uint32_t* ring_mine = reinterpret_cast<uint32_t*>(L.ring[h]);
    const uint32_t* ring_a = reinterpret_cast<const uint32_t*>(L.ring[0]);
    const uint32_t* ring_b = reinterpret_cast<const uint32_t*>(L.ring[1]);
    // ring slots of the given kind for MB x (see rg_kind)
    auto feed_ring = [&](int x, bool left) {
#pragma unroll
        for (int it = 0; it < 2; ++it) {
            const int k = rg_kind[it];
            if (left ? k == 1 : (k == 0 || (k == 2 && x == W - 1))) {
                const int ent = k == 1 ? (x + DRING - 1) & (DRING - 1) : x & (DRING - 1);
                ring_mine[ent * 32 + rg_dst[it]] = Sw[rg_src[it]];
            }
        }
    };

    prefetch(0);
    TRACE(const unsigned long long tr_first = __builtin_amdgcn_s_memrealtime();)
    for (int t = 0; t < steps; ++t) {
        const int x = t - h;
        const bool act = half_on && x >= 0 && x < W;
        const bool xl = x > 0, xr = x == W - 1;
        TRACE(unsigned long long ta = __builtin_amdgcn_s_memtime();)
        if (rp > 0) load_top(x);

        // ---- assemble the MB's own rows (an idle half scribbles on its own tiles only)
        Sw[a_y0] = pf_y0;
        Sw[a_y1] = pf_y1;
        Sw[a_c] = pf_c;
        if (hl < DBINFO_DWORDS) S.info[hl] = pf_i;
        // a band that starts below row 0 must not be filtered across its top edge (idc 1 or
        // a slice edge with idc 2): its top-edge strengths (bs[16..19] = info dword 4) are 0
        if (r == R0 && R0 > 0 && act && hl == 4 && pf_i != 0)
            __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t + 1 < steps) prefetch(t + 1);
        wave_sync();
        TRACE({ asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); const unsigned long long t2 = __builtin_amdgcn_s_memtime(); tph[0] += t2 - ta; tm = t2; })

        // ---- vertical edges of both halves (deblock.cc:488-504)
        filter_pass(S, hl, 0);
        wave_sync();
        // MB x-1's columns 12..15 (the left strip) are final for this row now: its ring entry
        // is complete
        if (act && xl && (feeds_ring || feeds_hb)) feed_ring(x, true);
        TRACE({ asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); const unsigned long long t2 = __builtin_amdgcn_s_memtime(); tph[1] += t2 - tm; tm = t2; })

        // ---- the record of the MB above (half A below another pair): wait for this epoch
        if (rp > 0) {
            const bool need = act && h == 0;
            WaitClock wc;
            TRACE(unsigned long long tw0 = 0;)
            while (!__all(!need || (top & 0xFFFFFFFF00000000ull) == tag)) {
                TRACE(if (!tw0) tw0 = __builtin_amdgcn_s_memrealtime();)
                __builtin_amdgcn_s_sleep(1);
                if (need) top = ld_cc64(hb_in + (size_t)x * 32 + hl);
                if (wait_give_up(err, wc)) {                     // bounded (device_common.h)
                    ok = false;
                    break;
                }
            }
            TRACE(if (tw0) tr_wait += __builtin_amdgcn_s_memrealtime() - tw0;)
            if (!ok) break;
        }
        wave_sync();
        TRACE(tm = __builtin_amdgcn_s_memtime();)
        // ---- the rows above: half A from the record, half B from half A's ring entry x
        // (A's MB x: columns 0..11 after H(x), 12..15 after V(x+1), this step)
        if (r > R0) Sw[a_top] = h == 0 ? (uint32_t)top : ring_a[(x & (DRING - 1)) * 32 + hl];
        // half B: the record of MB x-1 is complete
        if (act && feeds_hb && xl) st_rec(hb_out + (size_t)(x - 1) * 32 + hl, tag | ring_b[((x + DRING - 1) & (DRING - 1)) * 32 + hl], local);
        wave_sync();

        // ---- horizontal edges of both halves (deblock.cc:506-535)
        filter_pass(S, hl, 1);
        wave_sync();
        TRACE({ asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); const unsigned long long t2 = __builtin_amdgcn_s_memtime(); tph[2] += t2 - tm; tm = t2; })

        // ---- write back what is final (see the header comment)
#pragma unroll
        for (int it = 0; it < NWB; ++it) {
            const int f = wb_flags[it];
            const bool v = act && (f & 1) && (xl || !(f & 2)) && (xr || !(f & 4));
            if (v) *reinterpret_cast<uint32_t*>(wb_ptr[it] + x * ((f & 8) ? 8 : 16)) = Sw[wb_word[it]];
        }
        // ---- bottom rows of MB x, columns 0..11 (all 16 at the row end), into this half's ring
        if (act && (feeds_ring || feeds_hb)) feed_ring(x, false);
        wave_sync();
        // ---- half B at the row end: the last record
        if (act && feeds_hb && xr) st_rec(hb_out + (size_t)x * 32 + hl, tag | ring_b[(x & (DRING - 1)) * 32 + hl], local);
        // ---- carry the right 4 columns into the left strip of the next tile
#pragma unroll
        for (int it = 0; it < 2; ++it)
            if (cy_dst[it] >= 0) Sw[cy_dst[it]] = Sw[cy_src[it]];
        wave_sync();
        TRACE({ unsigned long long t2 = __builtin_amdgcn_s_memtime(); tph[3] += t2 - tm; })
    }
    if (!ok && feeds_hb)                                   // release the pair below (the error is flagged)
        for (int x = 0; x < W; ++x) st_rec(hb_out + (size_t)x * 32 + hl, tag, local);
    TRACE(if (lane == 0 && ticket < (1 << 16)) {
        h264r_db_trace[ticket][0] = tr_start; h264r_db_trace[ticket][1] = tr_first;
        h264r_db_trace[ticket][2] = __builtin_amdgcn_s_memrealtime(); h264r_db_trace[ticket][3] = tr_wait;
        for (int i = 0; i < 4; ++i) h264r_db_trace[ticket][4 + i] = tph[i]; })
    }
}
