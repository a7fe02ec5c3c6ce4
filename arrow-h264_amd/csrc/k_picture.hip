// k_picture.hip -- the order-dependent part of each picture: intra MBs and the
// loop filter.
//
// Intra prediction reads unfiltered neighbours of the current picture
// (intra_prediction.cc:140-186) and the loop filter runs MB by MB in raster
// order (deblock.cc:547-551); both make MB (x,y) depend on (x-1,y), (x,y-1) and
// (x+1,y-1): a wavefront with a 2-MB lag per row.
//
// A picture is cut into bands of <= 16 MB rows; one 1024-thread workgroup owns a
// band and each wave owns one row, walking it left to right.  Inside a band the
// row-to-row hand-off is an LDS counter with workgroup-scope release/acquire
// (no inter-CU traffic).  Only the first row of a band waits on another
// workgroup (the last row of the band above), through a progress counter in
// global memory published with agent-scope release every PUB MBs
// (MI355X_MICROARCH.md, Guideline 16 recipe).  Workgroups take (band, picture)
// tickets in band-major order from an atomic counter, so every workgroup only
// ever waits on a ticket taken earlier by a resident workgroup: no deadlock
// whatever the dispatch order or residency.  Every wait is bounded.
#include "mb_recon.h"
#include "mb_deblock.h"

using namespace h264r;

namespace {

constexpr int WAVES = 16;                   // rows per band
constexpr int PUB = 4;                      // global publish granularity (MBs)
constexpr unsigned SPIN_LIMIT = 1u << 24;   // bounded wait, then flag an error

DEV void publish_lds(int* counter, int value, int lane)
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // this wave's global stores are done
    if (lane == 0) __hip_atomic_store(counter, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

DEV void publish_global(int* counter, int value, int lane)
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");       // write back this XCD's dirty lines
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(counter, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool GLOBAL>
DEV bool wait_for(int* counter, int need, int* err)
{
    unsigned spins = 0;
    for (;;) {
        int v = GLOBAL ? __hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : __hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (v >= need) break;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > SPIN_LIMIT) {
            __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
    }
    if (GLOBAL) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    return true;
}

}  // namespace

// sync: [0] ticket counter, [1 ..] per (picture, row) progress; zeroed before every launch.
template <int PHASE, typename Scratch>
DEV void picture_walk(const h264r_batch& b, const DbInfo* dbinfo, int* sync, int* err, Scratch* scratch,
                      int* lprog, int* ticket_lds)
{
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int nbands = (g.hmb + WAVES - 1) / WAVES;
    const int bh = (g.hmb + nbands - 1) / nbands;            // rows per band (<= 16)
    if (threadIdx.x == 0) *ticket_lds = atomicAdd(&sync[0], 1);
    if (threadIdx.x < WAVES) lprog[threadIdx.x] = 0;
    __syncthreads();
    const int ticket = *ticket_lds;
    const int band = ticket / b.num_pics, pic = ticket % b.num_pics;
    const int r0 = band * bh, r1 = min(g.hmb, r0 + bh);
    const int r = r0 + wave;
    if (r >= r1) return;
    int* gprog = sync + 1 + (size_t)pic * g.hmb;
    const bool last_row = r == r1 - 1 && r1 < g.hmb;
    Scratch& S = scratch[wave];
    const h264r_mb* mbs = b.mbs + (size_t)pic * g.nmb;
    bool ok = true;

    for (int x = 0; x < g.wmb && ok; ++x) {
        const int need = min(x + 2, g.wmb);
        bool work = true;
        if constexpr (PHASE == 1) {
            const uint32_t w0 = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const uint32_t*>(&mbs[r * g.wmb + x]));
            work = ((w0 >> 8) & H264R_MBF_INTRA) && (w0 & 255) != H264R_I_PCM;
        }
        if (work && r > 0) {
            if (wave == 0) ok = wait_for<true>(&gprog[r - 1], need, err);
            else ok = wait_for<false>(&lprog[wave - 1], need, err);
        }
        if (work && ok) {
            if constexpr (PHASE == 1) intra_mb(b, g, pic, x, r, lane, S);
            else deblock_mb(b, g, pic, x, r, lane, S, dbinfo);
        }
        if (last_row) {
            if ((x + 1) % PUB == 0 || x + 1 == g.wmb) publish_global(&gprog[r], x + 1, lane);
        } else {
            publish_lds(&lprog[wave], x + 1, lane);
        }
    }
    if (!ok) {   // let every waiter behind a failed wave finish (outputs are flagged invalid)
        if (last_row) publish_global(&gprog[r], g.wmb, lane);
        else publish_lds(&lprog[wave], g.wmb, lane);
    }
}

extern "C" __global__ __launch_bounds__(1024) void k_intra_pic(h264r_batch b, int* sync, int* err)
{
    __shared__ IntraLds scratch[WAVES];
    __shared__ int lprog[WAVES];
    __shared__ int ticket;
    picture_walk<1>(b, nullptr, sync, err, scratch, lprog, &ticket);
}

// ---------------------------------------------------------------------------------
// Deblocking walk of one MB row by one wave.  The wave keeps the row's state in
// LDS: the left 4 columns carry over from the previous MB, the 4 rows above come
// from the ring of the wave above (same workgroup) or, for a band's first row,
// from global memory behind an agent-scope acquire; the next MB's samples and
// deblocking record are prefetched into registers while the current MB filters.
// Samples are written back as soon as no later MB of the raster order can modify
// them: rows 0..12 (chroma 0..4) by this wave, rows 13..15 (5..7) by the wave of
// the row below after its top-edge filtering, so no two waves ever store the
// same bytes inside a band and no global round trip sits on the in-band path.
// ---------------------------------------------------------------------------------
struct RowCtx {
    int r, wave, lane;
    bool band_top;        // first row of a band below another band: top rows from global
    bool has_consumer;    // a row below in this band reads our ring
    bool global_pub;      // last row of a band with a band below: publish to global
    bool write_bottom;    // rows 13..15 are written by us (no consumer in this band)
};

DEV void deblock_row(const h264r_batch& b, const DbInfo* __restrict__ dbinfo, const Geom& g, int pic,
                     const RowCtx& c, DbLds* scratch, int* lprog, int* gprog, int* err)
{
    const int lane = c.lane, r = c.r, W = g.wmb;
    DbLds& S = scratch[c.wave];
    uint8_t* Y = b.out_y + (size_t)pic * g.ysz;
    uint8_t* Cp[2] = {b.out_u + (size_t)pic * g.csz, b.out_v + (size_t)pic * g.csz};
    const int Y0 = r * 16, Yc = r * 8;
    const uint32_t* info_row = reinterpret_cast<const uint32_t*>(dbinfo + (size_t)pic * g.nmb + (size_t)r * W);
    // per-lane roles
    const int ly = lane >> 2, ld = lane & 3;                       // luma body dword
    const int cpl = (lane >> 4) & 1, cy = (lane >> 1) & 7, cd = lane & 1;   // chroma body dword (lanes 0..31)
    uint32_t pf_y = 0, pf_c = 0, pf_i = 0;
    auto prefetch = [&](int x) {
        pf_y = *reinterpret_cast<const uint32_t*>(Y + (size_t)(Y0 + ly) * g.W + x * 16 + 4 * ld);
        if (lane < 32) pf_c = *reinterpret_cast<const uint32_t*>(Cp[cpl] + (size_t)(Yc + cy) * g.Wc + x * 8 + 4 * cd);
        if (lane < 12) pf_i = info_row[x * 12 + lane];
    };
    prefetch(0);
    bool ok = true;
    for (int x = 0; x < W && ok; ++x) {
        const int X0 = x * 16, Xc = x * 8;
        if (r > 0) {
            if (c.band_top) ok = wait_for<true>(&gprog[r - 1], min(x + 2, W), err);
            else ok = wait_for<false>(&lprog[c.wave - 1], min(x + 2, W), err);
        }
        if (ok && c.has_consumer && x - RING + 1 > 0) ok = wait_for<false>(&lprog[c.wave + 1], x - RING + 1, err);
        if (!ok) break;
        // ---- assemble the tile: body (prefetched), record, top rows (left strip is the carry)
        S.lt[(4 + ly) * 5 + 1 + ld] = pf_y;
        if (lane < 32) S.ct[cpl][(4 + cy) * 3 + 1 + cd] = pf_c;
        if (lane < 8) reinterpret_cast<uint32_t*>(S.bs)[lane] = pf_i;
        else if (lane < 12) S.tail[lane - 8] = pf_i;
        if (r > 0) {
            if (c.band_top) {
                if (lane < 16)
                    S.lt[ly * 5 + 1 + ld] = *reinterpret_cast<const uint32_t*>(Y + (size_t)(Y0 - 4 + ly) * g.W + X0 + 4 * ld);
                else if (lane < 32) {
                    const int k = lane - 16, pl = k >> 3, i = (k >> 1) & 3, d = k & 1;
                    S.ct[pl][i * 3 + 1 + d] = *reinterpret_cast<const uint32_t*>(Cp[pl] + (size_t)(Yc - 4 + i) * g.Wc + Xc + 4 * d);
                }
            } else {
                const RingEntry& e = scratch[c.wave - 1].ring[x % RING];
                if (lane < 16) S.lt[ly * 5 + 1 + ld] = e.y[ly][ld];
                else if (lane < 32) {
                    const int k = lane - 16, pl = k >> 3, i = (k >> 1) & 3, d = k & 1;
                    S.ct[pl][i * 3 + 1 + d] = e.c[pl][i][d];
                }
            }
        }
        if (x + 1 < W) prefetch(x + 1);
        wave_sync();
        filter_mb(S, lane);

        // ---- write back what is final (see header comment)
        if (lane < 39) {                                   // luma rows 0..12, cols 0..11 of MB x
            const int row = lane / 3, d = 1 + lane % 3;
            *reinterpret_cast<uint32_t*>(Y + (size_t)(Y0 + row) * g.W + X0 + 4 * (d - 1)) = S.lt[(4 + row) * 5 + d];
        } else if (lane < 52) {                            // luma rows 0..12, cols 12..15 of MB x-1
            const int row = lane - 39;
            if (x > 0) *reinterpret_cast<uint32_t*>(Y + (size_t)(Y0 + row) * g.W + X0 - 4) = S.lt[(4 + row) * 5];
        } else if (r > 0) {                                // rows 13..15 of the row above, cols 0..15
            const int k = lane - 52, i = k >> 2, d = 1 + (k & 3);
            *reinterpret_cast<uint32_t*>(Y + (size_t)(Y0 - 3 + i) * g.W + X0 + 4 * (d - 1)) = S.lt[(1 + i) * 5 + d];
        }
        if (lane < 10) {                                   // chroma rows 0..4 cols 0..3 of MB x
            const int pl = lane / 5, row = lane % 5;
            *reinterpret_cast<uint32_t*>(Cp[pl] + (size_t)(Yc + row) * g.Wc + Xc) = S.ct[pl][(4 + row) * 3 + 1];
        } else if (lane < 20) {                            // chroma rows 0..4 cols 4..7 of MB x-1
            const int pl = (lane - 10) / 5, row = (lane - 10) % 5;
            if (x > 0) *reinterpret_cast<uint32_t*>(Cp[pl] + (size_t)(Yc + row) * g.Wc + Xc - 4) = S.ct[pl][(4 + row) * 3];
        } else if (lane < 32 && r > 0) {                   // chroma rows 5..7 of the row above
            const int k = lane - 20, pl = k / 6, i = (k % 6) >> 1, d = 1 + (k & 1);
            *reinterpret_cast<uint32_t*>(Cp[pl] + (size_t)(Yc - 3 + i) * g.Wc + Xc + 4 * (d - 1)) = S.ct[pl][(1 + i) * 3 + d];
        }
        if (c.write_bottom) {
            if (lane < 12) {                               // luma rows 13..15: MB x cols 0..11, MB x-1 cols 12..15
                const int i = lane >> 2, d = lane & 3;
                if (d > 0 || x > 0)
                    *reinterpret_cast<uint32_t*>(Y + (size_t)(Y0 + 13 + i) * g.W + X0 + 4 * (d - 1)) = S.lt[(17 + i) * 5 + d];
            } else if (lane < 24) {                        // chroma rows 5..7: MB x cols 0..3, MB x-1 cols 4..7
                const int k = lane - 12, pl = k / 6, i = (k % 6) >> 1, d = k & 1;
                if (d > 0 || x > 0)
                    *reinterpret_cast<uint32_t*>(Cp[pl] + (size_t)(Yc + 5 + i) * g.Wc + Xc + 4 * (d - 1)) = S.ct[pl][(9 + i) * 3 + d];
            }
        }
        if (x == W - 1) {                                  // end of row: cols 12..15 (chroma 4..7) of MB x
            const int nl = c.write_bottom ? 16 : 13, nc = c.write_bottom ? 8 : 5;
            if (lane < nl)
                *reinterpret_cast<uint32_t*>(Y + (size_t)(Y0 + lane) * g.W + X0 + 12) = S.lt[(4 + lane) * 5 + 4];
            else if (lane >= 32 && lane < 32 + 2 * nc) {
                const int k = lane - 32, pl = k / nc, row = k % nc;
                *reinterpret_cast<uint32_t*>(Cp[pl] + (size_t)(Yc + row) * g.Wc + Xc + 4) = S.ct[pl][(4 + row) * 3 + 2];
            }
        }
        // ---- ring for the row below: MB x cols 0..11 now, MB x-1 cols 12..15 now
        if (c.has_consumer) {
            RingEntry& e = S.ring[x % RING];
            RingEntry& ep = S.ring[(x + RING - 1) % RING];
            if (lane < 12) { const int i = lane / 3, d = lane % 3; e.y[i][d] = S.lt[(16 + i) * 5 + 1 + d]; }
            else if (lane < 16) { const int i = lane - 12; if (x > 0) ep.y[i][3] = S.lt[(16 + i) * 5]; }
            else if (lane < 24) { const int k = lane - 16, pl = k >> 2, i = k & 3; e.c[pl][i][0] = S.ct[pl][(8 + i) * 3 + 1]; }
            else if (lane < 32) { const int k = lane - 24, pl = k >> 2, i = k & 3; if (x > 0) ep.c[pl][i][1] = S.ct[pl][(8 + i) * 3]; }
            else if (x == W - 1) {
                if (lane < 36) { const int i = lane - 32; e.y[i][3] = S.lt[(16 + i) * 5 + 4]; }
                else if (lane < 44) { const int k = lane - 36, pl = k >> 2, i = k & 3; e.c[pl][i][1] = S.ct[pl][(8 + i) * 3 + 2]; }
            }
        }
        wave_sync();
        // ---- carry the right 4 columns into the left strip of the next tile
        if (lane < 20) S.lt[lane * 5] = S.lt[lane * 5 + 4];
        else if (lane < 44) { const int k = lane - 20, pl = k / 12, i = k % 12; S.ct[pl][i * 3] = S.ct[pl][i * 3 + 2]; }
        wave_sync();
        // ---- progress
        if (lane == 0) __hip_atomic_store(&lprog[c.wave], x + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (c.global_pub && ((x + 1) % PUB == 0 || x + 1 == W)) publish_global(&gprog[r], x + 1, lane);
    }
    if (!ok) {   // release every waiter behind a failed wave (the error word is set)
        if (lane == 0) __hip_atomic_store(&lprog[c.wave], W, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (c.global_pub) publish_global(&gprog[r], W, lane);
    }
}

extern "C" __global__ __launch_bounds__(1024) void k_deblock_pic(h264r_batch b, const DbInfo* dbinfo, int* sync, int* err)
{
    __shared__ DbLds scratch[WAVES];
    __shared__ int lprog[WAVES];
    __shared__ int ticket_lds;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int nbands = (g.hmb + WAVES - 1) / WAVES;
    const int bh = (g.hmb + nbands - 1) / nbands;
    if (threadIdx.x == 0) ticket_lds = atomicAdd(&sync[0], 1);
    if (threadIdx.x < WAVES) lprog[threadIdx.x] = 0;
    __syncthreads();
    const int ticket = ticket_lds;
    const int band = ticket / b.num_pics, pic = ticket % b.num_pics;
    const int r0 = band * bh, r1 = min(g.hmb, r0 + bh);
    RowCtx c;
    c.r = r0 + wave; c.wave = wave; c.lane = lane;
    if (c.r >= r1) return;
    c.band_top = wave == 0 && c.r > 0;
    c.has_consumer = c.r + 1 < r1;
    c.global_pub = c.r == r1 - 1 && r1 < g.hmb;
    c.write_bottom = !c.has_consumer;
    deblock_row(b, dbinfo, g, pic, c, scratch, lprog, sync + 1 + (size_t)pic * g.hmb, err);
}
