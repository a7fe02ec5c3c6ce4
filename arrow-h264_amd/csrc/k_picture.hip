// k_picture.hip -- intra MBs: the order-dependent part of reconstruction.
//
// Intra prediction reads unfiltered neighbours of the current picture
// (intra_prediction.cc:140-186), so MB (x,y) depends on (x-1,y), (x,y-1) and
// (x+1,y-1): a wavefront with a 2-MB lag per row.
//
// A picture is cut into bands of <= 16 MB rows; one 1024-thread workgroup owns a
// band and each wave owns one row, walking it left to right.  Inside a band the
// row-to-row hand-off is an LDS counter with workgroup-scope release/acquire
// (no inter-CU traffic).  Only the first row of a band waits on another
// workgroup (the last row of the band above), through a progress counter in
// global memory published with agent-scope release after every intra MB
// (MI355X_MICROARCH.md, Guideline 16 recipe).  Workgroups take (band, picture)
// tickets in band-major order from an atomic counter, so every workgroup only
// ever waits on a ticket taken earlier by a resident workgroup: no deadlock
// whatever the dispatch order or residency.  Every wait is bounded.
#include "mb_recon.h"

using namespace h264r;

namespace {

constexpr int WAVES = 16;                   // rows per band
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
template <typename Scratch>
DEV void picture_walk(const h264r_batch& b, int* sync, int* err, Scratch* scratch,
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

    // Only intra MBs take part in the walk (inter and PCM MBs were reconstructed by
    // k_inter).  Progress of a row = index of its first intra MB not yet done (W when
    // none is left): MB x may start once the row above has progress >= x + 2.
    const h264r_mb* row = mbs + (size_t)r * g.wmb;
    auto next_intra = [&](int from) -> int {
        for (int c = from & ~63; c < g.wmb; c += 64) {
            const int m = c + lane;
            bool in = false;
            if (m >= from && m < g.wmb) {
                const uint32_t w0 = *reinterpret_cast<const uint32_t*>(&row[m]);
                in = ((w0 >> 8) & H264R_MBF_INTRA) && (w0 & 255) != H264R_I_PCM;
            }
            const uint64_t bits = __ballot(in);
            if (bits) return c + __builtin_ctzll(bits);
        }
        return g.wmb;
    };
    auto publish = [&](int v) {
        if (last_row) publish_global(&gprog[r], v, lane);
        else publish_lds(&lprog[wave], v, lane);
    };
    int x = next_intra(0);
    publish(x);
    while (x < g.wmb && ok) {
        if (r > 0) {
            const int need = min(x + 2, g.wmb);
            if (wave == 0) ok = wait_for<true>(&gprog[r - 1], need, err);
            else ok = wait_for<false>(&lprog[wave - 1], need, err);
        }
        if (!ok) break;
        intra_mb(b, g, pic, x, r, lane, S);
        x = next_intra(x + 1);
        publish(x);
    }
    if (!ok) publish(g.wmb);   // let every waiter behind a failed wave finish (outputs are flagged invalid)
}

extern "C" __global__ __launch_bounds__(1024) void k_intra_pic(h264r_batch b, int* sync, int* err)
{
    __shared__ IntraLds scratch[WAVES];
    __shared__ int lprog[WAVES];
    __shared__ int ticket;
    picture_walk(b, sync, err, scratch, lprog, &ticket);
}
