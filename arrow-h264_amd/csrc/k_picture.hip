// k_picture.hip -- intra MBs: the order-dependent part of reconstruction.
//
// Intra prediction reads unfiltered neighbours of the current picture
// (intra_prediction.cc:140-186), so MB (x,y) depends on (x-1,y), (x,y-1) and
// (x+1,y-1): a wavefront with a 2-MB lag per row.
//
// A picture is cut into bands of <= 8 MB rows (H264R_WALK_ROWS); one 512-thread workgroup
// owns a band and each wave owns one row, walking it left to right.  Inside a band the
// row-to-row hand-off is an LDS counter with workgroup-scope release/acquire
// (no inter-CU traffic).  Only the first row of a band waits on another
// workgroup (the last row of the band above), through a progress counter in
// global memory published with agent-scope release every `gstep` intra MBs
// (MI355X_MICROARCH.md, Guideline 16 recipe).  Workgroups take (band, picture)
// tickets in band-major order from an atomic counter, so every workgroup only
// ever waits on a ticket taken earlier by a resident workgroup: no deadlock
// whatever the dispatch order or residency.  Every wait is bounded.
#include "mb_intra.h"

// k_intra_levels' register budget: 6 waves/SIMD = 80 VGPRs, no spill (LDS allows 7; at the
// default budget it took 82 = 5 waves: config 3 intra 1.235 -> 1.21 ms, configs 4 / 5 within
// noise, profiles/r05_at_level_waves_ab.txt)
#ifndef H264R_LVL_WAVES
#define H264R_LVL_WAVES 6
#endif
#define H264R_LEVEL_MAX_MBS 65536           // k_level keeps a picture's intra bitmap in LDS
#define H264R_LEVEL_LISTS 64                // levels 1 .. this many get per-level MB lists
#ifndef H264R_INTRA_PAIRS
#define H264R_INTRA_PAIRS 1                 // k_intra_levels reconstructs pairable MBs two per wave (intra_pair_i4)
#endif
#ifdef H264R_TRACE_INTRA
#undef H264R_INTRA_PAIRS
#define H264R_INTRA_PAIRS 0                 // the trace times one MB per item
#endif
// Two lists per level: id 2 L = its pairable MBs (intra_pairable: I_4x4, not lossless), id
// 2 L + 1 the others, laid out in id order; count / base / cursor arrays of LEVEL_IDS ints.
constexpr int LEVEL_IDS = 2 * (H264R_LEVEL_LISTS + 1);

using namespace h264r;

#ifdef H264R_TRACE_INTRA
// per-MB trace (trace builds only: tools/trace_intra.py): {start, end} in 100 MHz ticks,
// [2] = level << 32 | mb_type (k_intra_levels) or 1 << 31 | wait ticks << 8 | mb_type (the
// walk: the wait for the row above, then the MB), [3] = phase cycles / 16 (16 bits each)
__device__ unsigned long long h264r_intra_trace[1 << 20][4];
__device__ unsigned h264r_intra_trace_n;
DEV void intra_trace_put(unsigned long long t0, unsigned long long w, const unsigned long long (&tph)[5], unsigned long long c0, int lane)
{
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (lane) return;
    const unsigned slot = atomicAdd(&h264r_intra_trace_n, 1u);
    if (slot >= (1u << 20)) return;
    unsigned long long ph = 0, prev = c0;
    for (int q = 0; q < 4; ++q) {
        ph |= (unsigned long long)min((tph[q] - prev) >> 4, 65535ull) << (16 * q);
        prev = tph[q];
    }
    h264r_intra_trace[slot][0] = t0; h264r_intra_trace[slot][1] = t1;
    h264r_intra_trace[slot][2] = w;
    h264r_intra_trace[slot][3] = ph;
}
#endif

namespace {

#ifndef H264R_WALK_ROWS
#define H264R_WALK_ROWS 8                   // MB rows per band (h264r_host.hip sizes the launch with it)
#endif
#ifndef H264R_WALK_WAVES
#define H264R_WALK_WAVES 8                  // minimum waves per SIMD asked of the register allocator (<= 64 VGPRs; profiles/r03s2_b_ab.txt)
#endif
constexpr int WAVES = H264R_WALK_ROWS;      // rows per band, one wave each

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

// seen: the progress value observed (and acquired); a later need <= seen needs no new wait:
// what was published before that value was visible after the acquire that followed it.
template <bool GLOBAL>
DEV bool wait_for(int* counter, int need, int* err, int& seen)
{
    WaitClock wc;
    for (;;) {
        int v = GLOBAL ? __hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : __hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        seen = v;
        if (v >= need) break;
        __builtin_amdgcn_s_sleep(1);
        if (wait_give_up(err, wc)) return false;     // bounded (device_common.h)
    }
    if (GLOBAL) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    return true;
}

}  // namespace

// One (band, picture) ticket: wave `wave` walks MB row r0 + wave of the band.
// sync: [0] ticket counter, [1 ..] per (picture, row) progress; zeroed before every launch.
// Bit `band` of a picture's band mask (k_level: bit b for band b; all bits set, or none, when the
// picture has more than 31 bands -- a shift by 32 or more is not defined in C++)
DEV bool band_bit(int pb, int band) { return band >= 32 ? pb != 0 : ((pb >> band) & 1) != 0; }

// pband[pic] (with lvl): bit b set when band b of the picture has an MB deeper than lmax
// (k_level); a band without one needs no walk, and the band below it no wait.
template <typename Scratch>
DEV void walk_ticket(const h264r_batch& b, int* sync, int* err, Scratch* scratch, const uint32_t* tap4, int* lprog, int ticket,
                     const uint16_t* __restrict__ lvl, int lmax, int2 rows, int gstep, uint8_t* recon, const int* pband)
{
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int R0 = rows.x, R1 = rows.y, HB = R1 - R0;         // MB rows of this launch
    const int nbands = (HB + WAVES - 1) / WAVES;
    const int bh = (HB + nbands - 1) / nbands;               // rows per band (<= WAVES)
    const int band = ticket / b.num_pics, pic = ticket % b.num_pics;
    const int r0 = R0 + band * bh, r1 = min(R1, r0 + bh);
    const int r = r0 + wave;
    if (r >= r1) return;
    // the band above has nothing deeper than the lists: its rows are final already
    const bool above_done = lvl && band > 0 && !band_bit(pband[pic], band - 1);
    int* gprog = sync + 1 + (size_t)pic * g.hmb;
    const bool last_row = r == r1 - 1 && r1 < R1;
    Scratch& S = scratch[wave];
    const h264r_mb* mbs = b.mbs + (size_t)pic * g.nmb;
    bool ok = true;

    // Only intra MBs take part in the walk (inter and PCM MBs were reconstructed by
    // k_inter).  Progress of a row = index of its first intra MB not yet done (W when
    // none is left): MB x may start once the row above has progress >= x + 2.
    const h264r_mb* row = mbs + (size_t)r * g.wmb;
    const uint16_t* lrow = lvl ? lvl + (size_t)pic * g.nmb + (size_t)r * g.wmb : nullptr;
    // (the row's intra bits are loaded once per 64-MB chunk and kept: records are immutable
    // during a batch, so the walk does not reload them after every MB)
    int cbase = -64;
    uint64_t cbits = 0;
    auto next_intra = [&](int from) -> int {
        for (int c = from & ~63; c < g.wmb; c += 64) {
            if (c != cbase) {
                const int m = c + lane;
                bool in = false;
                if (m < g.wmb) {
                    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(&row[m]);
                    in = ((w0 >> 8) & H264R_MBF_INTRA) && (w0 & 255) != H264R_I_PCM;
                    if (lrow && lrow[m] <= lmax) in = false;      // done by k_intra_lvl
                }
                cbits = __ballot(in);
                cbase = c;
            }
            const uint64_t bits = from > c ? cbits & (~0ull << (from - c)) : cbits;
            if (bits) return c + __builtin_ctzll(bits);
        }
        return g.wmb;
    };
    // The band's last row publishes to the next band through global memory, an agent-scope
    // release (L2 write-back of the XCD's dirty lines) each time: every `gstep` MBs and at
    // the row end.  With band-major tickets the next band of a picture comes a batch's worth
    // of tickets later, so large batches take a coarse gstep (the next band's first row is
    // not waiting; one release per MB on every band's last row cost config 2 a quarter of its
    // walk time, profiles/r02_intra_walk_gstep.txt), small ones 1.
    // A row that stored nothing since its last global publish (no intra MB) skips the
    // release: the relaxed flag store alone.
    int gpub = -1;
    bool dirty = false;
    auto publish = [&](int v, bool force) {
        if (last_row) {
            if (force || v >= g.wmb || v - gpub >= gstep) {
                if (dirty) publish_global(&gprog[r], v, lane);
                else if (lane == 0) __hip_atomic_store(&gprog[r], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                gpub = v;
                dirty = false;
            }
        } else {
            publish_lds(&lprog[wave], v, lane);
        }
    };
    int x = next_intra(0);
    publish(x, true);
    int seen = 0;                                            // progress of the row above, acquired
    while (x < g.wmb && ok) {
        // the lane, opaque per MB: what derives from it is recomputed per MB, not hoisted out of
        // the walk and kept live across it
        int ln = lane;
        asm volatile("" : "+v"(ln));
        // the MB's records and levels do not depend on the row above: in flight during the wait
        IntraHead hd;
        intra_head_records(b, g, pic, x, r, ln, hd);
        const IntraLoads ld = intra_body_loads(b, pic, hd, ln);
        // gstep < 0: the host's wait test (H264R_DBG_WAIT_TEST) -- a need no row ever meets
        const int need = gstep < 0 ? g.wmb + 1 : min(x + 2, g.wmb);
#ifdef H264R_TRACE_INTRA
        const unsigned long long t_wait0 = __builtin_amdgcn_s_memrealtime();
#endif
        if (r > R0 && need > seen && !(wave == 0 && above_done)) {
            if (wave == 0) ok = wait_for<true>(&gprog[r - 1], need, err, seen);
            else ok = wait_for<false>(&lprog[wave - 1], need, err, seen);
        }
        if (!ok) break;
        hd.nb = intra_head_samples(g, pic, x, r, ln, recon, tap4);
#ifdef H264R_TRACE_INTRA
        {
            const unsigned long long tw = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
            unsigned long long tph[5] = {c0, c0, c0, c0, c0};
            intra_mb_compute(b, g, pic, x, r, ln, S, tap4, hd, ld, recon, tph);
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            const unsigned long long wait = min((tw - t_wait0) , 0xFFFFFull);
            intra_trace_put(t_wait0, (1ull << 31) | (wait << 8) | (unsigned)row[x].mb_type, tph, c0, lane);
        }
#else
        intra_mb_compute(b, g, pic, x, r, ln, S, tap4, hd, ld, recon);
#endif
        dirty = true;
        x = next_intra(x + 1);
        publish(x, false);
    }
    if (!ok) { dirty = true; publish(g.wmb, true); }   // let every waiter behind a failed wave finish (outputs are flagged invalid)
}

// lvl / lmax: intra MBs with lvl <= lmax were reconstructed by the k_intra_lvl
// launches before this one (lvl == nullptr: the walk does every intra MB).
// pband[pic] (k_level): the picture's bands with an MB deeper than lmax (all for a picture left
// to the walk whole) -- a band without one has nothing here, and its ticket returns.
extern "C" __global__ __launch_bounds__(64 * H264R_WALK_ROWS, H264R_WALK_WAVES) void k_intra_pic(h264r_batch b, int* sync, int* err,
                                                              const uint16_t* lvl, int lmax, int2 rows, int gstep,
                                                              uint8_t* recon, const int* pband)
{
    __shared__ IntraScratch scratch[WAVES];
    __shared__ uint32_t tap4[INTRA_TAPS];
    __shared__ int lprog[WAVES];
    __shared__ int ticket;
    if (threadIdx.x == 0) ticket = atomicAdd(&sync[0], 1);
    if (threadIdx.x < WAVES) lprog[threadIdx.x] = 0;
    __syncthreads();
    if (lvl && !band_bit(pband[ticket % b.num_pics], ticket / b.num_pics)) return;       // (block-uniform)
    intra4_tap_fill(tap4, threadIdx.x, blockDim.x);
    __syncthreads();
    walk_ticket(b, sync, err, scratch, tap4, lprog, ticket, lvl, lmax, rows, gstep, recon, pband);
}

// ------------------------------------------------------------ level schedule
// An intra MB reads the unfiltered samples of its neighbours A (x-1,y), B (x,y-1),
// C (x+1,y-1) and D (x-1,y-1) (intra_prediction.cc:140-186, 683-695, 806-823).
// Inter and I_PCM MBs are final after k_inter, so only intra -> intra edges
// order the work: level(MB) = 0 for inter / I_PCM, else 1 + max(level of A, B, C,
// D) (out of picture = 0).  Every MB of level L depends only on levels < L, so
// one launch per level needs no in-kernel synchronisation at all.  In P / B
// pictures (10 % intra MBs) the deepest chain is a handful of levels; in all-intra
// pictures level(x, y) = x + 2y + 1 and the levels beyond `lmax` fall back to the
// wavefront walk (k_intra_pic).  Slice boundaries are ignored here: that can only
// raise a level, never break an order.
//
// k_level: one 1024-thread workgroup per picture, the levels relaxed in LDS.  Its threads load
// the picture's intra and pairable bits, then iterate L(m) = intra(m) ? 1 + max(L(A), L(B),
// L(C), L(D)) : 0 over all MBs in place (levels as bytes, a zero border around the rows), from
// L = 1 on every intra MB, until a pass changes nothing.  The values only grow and never pass
// the true level (a chaotic relaxation of a monotone map on a DAG, so in-place races are
// harmless): after k passes every MB of level <= k + 1 is exact, so a picture converges in
// (deepest level) + 1 passes -- about 8 in the P / B pictures of the benchmark -- and a picture
// still changing after deep_cut + 1 passes is deeper than deep_cut (all-intra) and goes to the
// walk whole.  It replaced a walk of the rows in lock step (one thread per row, one workgroup
// barrier per MB step, x + 2y steps): 88 us per 1080p picture in the latency chain, 148 us per
// 1024-picture batch (profiles/r05_ac_latency_kernels.txt, r04_ak_kernel_stats_b1024.csv).
// lcount[id] (id 2 L + c, L = 1 .. H264R_LEVEL_LISTS, c = 0 pairable): intra MBs of level L over
// the batch (zeroed per batch); k_level_scatter turns them into the lists.
constexpr int LEVEL_LDS = 40960;            // (W + 2) x (rows + 1) level bytes (h264r_host.hip checks)
extern "C" __global__ __launch_bounds__(1024) void k_level(h264r_batch b, uint16_t* lvl, int* lvsync, int* lcount, int2 rows,
                                                          int deep_cut, int lmax, int* pband)
{
    __shared__ uint64_t bits[H264R_LEVEL_MAX_MBS / 64];   // intra (not PCM) MBs of the picture
    __shared__ uint64_t pbits[H264R_LEVEL_MAX_MBS / 64];  // the pairable ones among them
    __shared__ uint8_t lv[LEVEL_LDS];                     // level of band row r, MB x at (r + 1) * (W + 2) + x + 1
    __shared__ int hist[LEVEL_IDS];
    __shared__ int pdeep, sband;
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int pic = blockIdx.x, tid = threadIdx.x, lane = tid & 63, nt = (int)blockDim.x;
    const h264r_mb* mbs = b.mbs + (size_t)pic * g.nmb;
    const int R0 = rows.x, HB = rows.y - rows.x, W = g.wmb, P = W + 2, n = HB * W;   // rows above R0 count as level 0
    for (int i = tid; i < LEVEL_IDS; i += nt) hist[i] = 0;
    for (int i = tid; i < P * (HB + 1); i += nt) lv[i] = 0;
    if (tid == 0) { pdeep = 0; sband = 0; }
    // the walk's bands (walk_ticket): bit b of pband for band b, all bits past 31 bands
    const int wb = (HB + WAVES - 1) / WAVES, wbh = (HB + wb - 1) / wb;
    constexpr int UNR = 4;                                 // record loads in flight per thread
    for (int base = 0; base < n; base += UNR * nt) {
        uint32_t w0[UNR];
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
            const int m = base + k * nt + tid;
            w0[k] = m < n ? *reinterpret_cast<const uint32_t*>(&mbs[R0 * W + m]) : 0u;
        }
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
            const int m = base + k * nt + tid;
            const bool in = ((w0[k] >> 8) & H264R_MBF_INTRA) && (w0[k] & 255) != H264R_I_PCM;
            const bool pr = in && (w0[k] & 255) == H264R_I_4x4 && !((w0[k] >> 8) & H264R_MBF_BYPASS);   // intra_pairable
            const uint64_t bl = __ballot(in), pl = __ballot(pr);
            if (lane == 0 && m < n) {
                bits[m >> 6] = bl;
                pbits[m >> 6] = pl;
            }
        }
    }
    __syncthreads();
    // this thread's MBs m = tid + k nt as LDS byte indices, stepped without a division per MB
    const int dr = nt / W, dx = nt % W, r0 = tid / W, x0 = tid % W;
    auto lds_index = [&](int& r, int& x) {
        const int i = (r + 1) * P + x + 1;
        x += dx; r += dr;
        if (x >= W) { x -= W; ++r; }
        return i;
    };
    // L = 1 on every intra MB, then passes until nothing changes (or the picture proves deep)
    {
        int r = r0, x = x0;
        for (int m = tid; m < n; m += nt) {
            const int i = lds_index(r, x);
            if ((bits[m >> 6] >> (m & 63)) & 1) lv[i] = 1;
        }
    }
    const int cut = min(deep_cut, 250);                    // bytes: levels up to 251 are kept exact
    bool deep = true;
    for (int pass = 0; pass <= cut + 1; ++pass) {
        __syncthreads();
        int changed = 0;
        int r = r0, x = x0;
        for (int m = tid; m < n; m += nt) {
            const int i = lds_index(r, x);
            if (!((bits[m >> 6] >> (m & 63)) & 1)) continue;
            const int v = 1 + max(max((int)lv[i - P - 1], (int)lv[i - P]), max((int)lv[i - P + 1], (int)lv[i - 1]));
            if (v != lv[i]) {
                lv[i] = (uint8_t)min(v, 255);
                changed = 1;
            }
        }
        if (!__syncthreads_or(changed)) { deep = false; break; }
    }
    // the levels out (uint16), the per-list counts, the deepest level
    int deepest = 0;
    if (!deep) {
        uint16_t* out = lvl + (size_t)pic * g.nmb + (size_t)R0 * W;
        int r = r0, x = x0;
        for (int m = tid; m < n; m += nt) {
            const int rr = r;                              // (lds_index steps r, x to the next MB)
            const int L = lv[lds_index(r, x)];
            out[m] = (uint16_t)L;
            deepest = max(deepest, L);
            if (L > lmax) atomicOr(&sband, wb > 31 ? -1 : 1 << (rr / wbh));
            if (L >= 1 && L <= H264R_LEVEL_LISTS) atomicAdd(&hist[2 * L + !((pbits[m >> 6] >> (m & 63)) & 1)], 1);
        }
        for (int d = 32; d >= 1; d >>= 1) deepest = max(deepest, __shfl_xor(deepest, d));
        if (lane == 0 && deepest) atomicMax(&pdeep, deepest);
    }
    __syncthreads();
    deepest = pdeep;
    // a picture deeper than deep_cut (all-intra: level x + 2y + 1) goes to the walk whole:
    // its few MBs per level would only make k_intra_levels wait at its grid barriers
    if (deep || deepest > deep_cut) {
        for (int m = R0 * W + tid; m < rows.y * W; m += nt) lvl[(size_t)pic * g.nmb + m] = 0xFFFF;
        if (tid == 0) pband[pic] = -1;
        return;
    }
    if (tid == 0) pband[pic] = sband;
    if (tid == 0 && deepest) atomicMax(&lvsync[1], deepest);
    for (int i = tid + 2; i < LEVEL_IDS; i += nt)
        if (hist[i]) atomicAdd(&lcount[i], hist[i]);
}

// The per-level MB lists: lbase[L] = exclusive prefix of lcount over levels (each
// k_level_scatter workgroup scans them itself), then every intra MB of level 1 .. H264R_LEVEL_LISTS appends
// pic * nmb + addr to its level's list (k_level_scatter: a workgroup counts its MBs per
// level in LDS and reserves each level's range with one global atomic).
// lcount, lbase, lcursor: LEVEL_IDS ints each.
// One workgroup per picture: an LDS count per level over the picture's MBs, one global
// atomic per (picture, level) to reserve its range, then the entries (a workgroup per
// 256 MBs reserved per (workgroup, level) instead: 130 k atomics on a few counters,
// 375 us per 1024 1080p pictures).
constexpr int SCATTER_PER = 16;             // MBs per thread (1024 threads: pictures up to 16 k MBs per pass)
// Every workgroup first scans the level counts itself (one wave, 3 ids a lane; workgroup 0
// stores the bases for k_intra_levels): a separate one-workgroup scan launch cost more.
extern "C" __global__ __launch_bounds__(1024) void k_level_scatter(h264r_batch b, const uint16_t* __restrict__ lvl,
                                                                   const int* __restrict__ lcount, int* lbase, int* lcursor,
                                                                   uint32_t* __restrict__ list, int2 rows)
{
    static_assert(LEVEL_IDS <= 3 * 64, "one wave scans the level counts");
    __shared__ int cnt[LEVEL_IDS];
    __shared__ int res[LEVEL_IDS];
    __shared__ int sbase[LEVEL_IDS];
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int pic = blockIdx.x, tid = threadIdx.x;
    if (tid < 64) {
        int v[3], sum = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            v[k] = 3 * tid + k < LEVEL_IDS ? lcount[3 * tid + k] : 0;
            sum += v[k];
        }
        int inc = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int up = __shfl_up(inc, o, 64);
            if (tid >= o) inc += up;
        }
        int run = inc - sum;
#pragma unroll
        for (int k = 0; k < 3; ++k)
            if (3 * tid + k < LEVEL_IDS) {
                sbase[3 * tid + k] = run;
                if (pic == 0) lbase[3 * tid + k] = run;
                run += v[k];
            }
    }
    const int m0 = rows.x * g.wmb, m1 = rows.y * g.wmb;
    const uint16_t* lp = lvl + (size_t)pic * g.nmb;
    const h264r_mb* mbs = b.mbs + (size_t)pic * g.nmb;
    for (int base = m0; base < m1; base += 1024 * SCATTER_PER) {
        if (tid < LEVEL_IDS) cnt[tid] = 0;
        __syncthreads();
        int L[SCATTER_PER], rank[SCATTER_PER];
#pragma unroll
        for (int k = 0; k < SCATTER_PER; ++k) {
            const int m = base + k * 1024 + tid;
            const int lv = m < m1 ? lp[m] : 0;
            // the list id: 2 L for a pairable MB (intra_pairable; k_level counted the same), else 2 L + 1
            const uint32_t w0 = lv >= 1 && lv <= H264R_LEVEL_LISTS ? *reinterpret_cast<const uint32_t*>(&mbs[m]) : 0u;
            const bool pr = (w0 & 255) == H264R_I_4x4 && !((w0 >> 8) & H264R_MBF_BYPASS);
            L[k] = lv >= 1 && lv <= H264R_LEVEL_LISTS ? 2 * lv + !pr : 0;
        }
#pragma unroll
        for (int k = 0; k < SCATTER_PER; ++k) rank[k] = L[k] ? atomicAdd(&cnt[L[k]], 1) : 0;
        __syncthreads();
        if (tid >= 2 && tid < LEVEL_IDS && cnt[tid]) res[tid] = atomicAdd(&lcursor[tid], cnt[tid]);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < SCATTER_PER; ++k)
            if (L[k]) list[sbase[L[k]] + res[L[k]] + rank[k]] = (uint32_t)((size_t)pic * g.nmb + base + k * 1024 + tid);
        __syncthreads();
    }
}

// k_intra_levels: the intra MBs of levels 1..min(lmax, deepest level), one level
// after the other inside one persistent launch (a launch per level would pay a cold
// instruction cache on every CU each time).  Every workgroup must be resident: the
// host sizes the grid from the occupancy query.  Levels are separated by a grid
// barrier: stores drained, agent release, then an arrival on one of 8 shard counters
// (workgroup b on shard b % 8, the XCD it was dispatched to); a shard's last arrival adds
// to the top counter (after an acquire-release fence: it carries its shard's releases)
// and every workgroup waits on the top counter, then acquires.  One counter for all the
// ~1000 arrivals had serialised them (MI355X_MICROARCH.md price list 'barrier-counter' vs
// 'barrier-xcd', 'fanin').  Each wave takes its level's items grid-stride.
// bar: [0..7] shard counters, [8] top counter, zeroed per batch (by k_inter4r); L = 1, 2, ...
DEV bool grid_barrier(int* bar, int L, int* err)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int ok;
    if (threadIdx.x == 0) {
        const int G = (int)gridDim.x, sh = (int)blockIdx.x & 7;
        const int nsh = (G - sh + 7) / 8, nshards = min(G, 8);           // workgroups of my shard; shards
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (__hip_atomic_fetch_add(&bar[sh], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == L * nsh - 1) {
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
            __hip_atomic_fetch_add(&bar[8], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        WaitClock wc;
        ok = 1;
        while (__hip_atomic_load(&bar[8], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < L * nshards) {
            __builtin_amdgcn_s_sleep(2);
            if (wait_give_up(err, wc)) { ok = 0; break; }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    return ok;
}

#ifdef H264R_TRACE_INTRA
extern "C" __global__ void k_intra_trace_dump(unsigned long long* out, unsigned* n)
{
    const unsigned cnt = h264r_intra_trace_n < (1u << 20) ? h264r_intra_trace_n : (1u << 20);
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x)
        for (int j = 0; j < 4; ++j) out[i * 4 + j] = h264r_intra_trace[i][j];
    if (blockIdx.x == 0 && threadIdx.x == 0) *n = cnt;
}
#endif

extern "C" __global__ __launch_bounds__(256, H264R_LVL_WAVES) void k_intra_levels(h264r_batch b, const int* __restrict__ lcount,
                                                                                const int* __restrict__ lbase,
                                                                                const uint32_t* __restrict__ list,
                                                                                int lmax, int* lvsync, int* err, uint8_t* recon,
                                                                                int* bar)
{
    __shared__ IntraScratch scratch[H264R_INTRA_PAIRS ? 8 : 4];
    __shared__ uint32_t tap4[INTRA_TAPS];
    intra4_tap_fill(tap4, threadIdx.x, blockDim.x);
    __syncthreads();
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int nw = (int)gridDim.x * 4, gw = (int)blockIdx.x * 4 + wave;
    const int deepest = __hip_atomic_load(&lvsync[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int top = min(lmax, deepest);
    for (int L = 1; L <= top; ++L) {
        // the MBs of level L, wave-strided over its items (entry = pic * nmb + addr): the pairs of
        // its pairable list, then one MB at a time the rest of it and the other list (the two
        // lists are consecutive)
        const int n0 = lcount[2 * L], n1 = lcount[2 * L + 1], base = lbase[2 * L];
        const int np = H264R_INTRA_PAIRS ? n0 / 2 : 0, items = n0 + n1 - np;
        for (int e = gw; e < items; e += nw) {
            int ln = lane;                                 // opaque per item (see walk_ticket)
            asm volatile("" : "+v"(ln));
            if (e < np) {
                // k_level and k_level_scatter classify as intra_pairable does: a pair that is not
                // one is a broken list, flagged as a device error (h264r_check)
                if (!intra_pair_i4(b, g, list[base + 2 * e], list[base + 2 * e + 1], ln, scratch[wave], scratch[4 + wave],
                                   tap4, recon))
                    __hip_atomic_store(err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                continue;
            }
            const uint32_t k = list[base + np + e];
            const int pic = (int)(k / (unsigned)g.nmb), a = (int)(k % (unsigned)g.nmb);
#ifdef H264R_TRACE_INTRA
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
            unsigned long long tph[5] = {c0, c0, c0, c0, c0};
            intra_mb2(b, g, pic, a % g.wmb, a / g.wmb, lane, scratch[wave], tap4, recon, tph);
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
            if (lane == 0) {
                const unsigned slot = atomicAdd(&h264r_intra_trace_n, 1u);
                if (slot < (1u << 20)) {
                    // [3]: core cycles / 16 of the phases (record, residual, tiles, prediction), 16 bits each
                    unsigned long long ph = 0, prev = c0;
                    for (int q = 0; q < 4; ++q) {
                        ph |= (unsigned long long)min((tph[q] - prev) >> 4, 65535ull) << (16 * q);
                        prev = tph[q];
                    }
                    h264r_intra_trace[slot][0] = t0; h264r_intra_trace[slot][1] = t1;
                    h264r_intra_trace[slot][2] = ((unsigned long long)L << 32) | (unsigned)(b.mbs[(size_t)pic * g.nmb + a].mb_type);
                    h264r_intra_trace[slot][3] = ph;
                }
            }
#else
            intra_mb2(b, g, pic, a % g.wmb, a / g.wmb, ln, scratch[wave], tap4, recon);
#endif
        }
        if (L < top && !grid_barrier(bar, L, err)) return;
    }
}
