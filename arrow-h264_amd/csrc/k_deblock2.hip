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
// into registers as 32-byte row pieces and stored back the same way, so global traffic
// stays in whole sectors (a lane-pair walk with 16-byte scattered accesses missed L2:
// profiles/r02_deblock2_v1_pmc_b256.txt).
//
// The row below needs each MB's bottom rows (luma 12..15, chroma 6..7) after the MB's
// right neighbour filtered its left edge: 24 naturally aligned 8-byte granules {data
// dword, tag} per MB, laid out so that lane q of the row below polls exactly the six
// it filters with (luma dword q of rows 12..15, chroma plane q/2 dword q&1 of rows 6..7)
// and the producing lane publishes exactly the six it holds after its horizontal pass
// -- no LDS exchange on either side.  Luma dword 3 and chroma dword 1 change again
// with MB x+1's vertical edges and are published after them.  Write-through `sc1`
// stores, `sc1` polling loads until every granule carries this launch's tag
// (MI355X_MICROARCH.md R2 granule hand-off).  Waves take tickets row-major, so a wave
// only waits on tickets taken earlier by running waves; every spin is bounded and
// flags the error word.
//
// Memory operations are issued in the order their waits need (vmcnt is in order and
// counts stores): the record loads first, then the next MB's DbInfo and the next
// window, whose registers are not needed before the end of the step (DbInfo goes
// through LDS, so no loaded register is carried into the next step's filters).
//
// Sample ownership (each sample stored once, when final): a row stores MB x's rows
// 0..12 (chroma 0..6) once MB x+1's vertical edges are done, and the rows 13..15
// (chroma 7) of MB (x, y-1) after filtering its own top edge.  The last row of the
// band stores its own bottom rows.
#include <type_traits>

#include "mb_deblock.h"
#include "mb_deblock2.h"

using namespace h264r;

namespace {

constexpr int UNITS = DEBLOCK2_UNITS;  // (picture, MB row) units per wave, 4 lanes each
constexpr int RECG = 24;               // granules per MB record: [consumer lane c 0..3][i 0..5]
constexpr int AUX_SC1 = 16;            // buffer-op cache policy: sc1 (write-through store, L2-served load)

// One unit's MB row in LDS (1264 B: a unit stride of 316 dwords spreads the 8 units of
// a half-wave over distinct banks for the column reads of the horizontal pass).
struct alignas(16) UnitLds {
    uint32_t y[16][12];       // luma rows 0..15; MB x in slot s = x % 3: dwords 4s .. 4s+3
    uint32_t c[2][8][6];      // chroma plane, rows 0..7; slot s = dwords 2s, 2s+1
    uint32_t info[20];        // DbInfo of the MB being filtered
    uint32_t pad[8];
};
static_assert(sizeof(UnitLds) == 1264, "UnitLds layout");

typedef uint32_t v4u __attribute__((ext_vector_type(4)));   // native vectors: registers, not stack
typedef uint32_t v2u __attribute__((ext_vector_type(2)));


// {byte j, byte j + 2} of one dword as an s16x2 (the column pair (j, j+2)).
DEV s2 unpack_cols(uint32_t w, int j) { return as_s2(__builtin_amdgcn_perm(w, w, 0x0C000C00u | ((uint32_t)(j + 2) << 16) | (uint32_t)j)); }
// Column pairs (0, 2) and (1, 3) back into one dword.
DEV uint32_t pack_cols(s2 c0, s2 c1) { return __builtin_amdgcn_perm(as_w(c1), as_w(c0), 0x06020400u); }
DEV s2 bs_pair(uint32_t w, int slo, int shi) { return (s2){(short)((w >> (8 * slo)) & 255), (short)((w >> (8 * shi)) & 255)}; }

}  // namespace

#ifdef H264R_TRACE
// Timing trace (trace builds only: make EXTRA=-DH264R_TRACE): per ticket {start, end
// (s_memrealtime, 100 MHz), then s_memtime cycles spent in: V pass, record wait,
// H pass, publish + stores + window switch}.
__device__ unsigned long long h264r_db2_trace[1 << 16][8];
#define TRACE(...) __VA_ARGS__
extern "C" void h264r_db2_trace_copy(void* dst) { (void)hipMemcpyFromSymbol(dst, HIP_SYMBOL(h264r_db2_trace), sizeof(h264r_db2_trace)); }
#else
#define TRACE(...)
#endif

// hb: records [pic][row & 1][W][RECG] granules {dword, tag}, moved as 16-byte `sc1` pairs
// (two granules; each 8-byte half observed untorn on gfx950, MI355X_MICROARCH.md
// visibility: the tag check stays per granule); sync[0]: ticket counter;
// epoch < 2^20 (the host restarts from zeroed records before it wraps).
// XCD-local hand-off (H264R_DB2_XCD, default): the rows of a 16-picture group all run on
// one XCD -- group g on XCD g % nx, each XCD with its own ticket counter (the XCD read
// from the hardware register, so the placement holds whatever the dispatch order) -- and
// the hand-off records are plain stores, which stay in that XCD's L2, read back by `sc1`
// loads (L1 bypassed, L2 hit) instead of write-through stores and loads served from the
// fabric.  Each wave takes tickets until its XCD's run out, so an XCD finishes its groups
// as long as any wave lands on it: the host asks for this mode (nx > 1) only for grids of
// >= 64 waves per XCD, rounded up to whole round-robin cycles.
#ifndef H264R_DB2_XCD
#define H264R_DB2_XCD 1
#endif
extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_deblock2(
    h264r_batch b, const DbInfo* __restrict__ dbinfo, uint64_t* hb, int* sync, int* err, uint32_t epoch, int2 rows, int nx,
    const uint8_t* __restrict__ recon)
{
    __shared__ UnitLds S[UNITS];
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int W = g.wmb, R0 = rows.x, R1 = rows.y;
    const int ngroups = (b.num_pics + UNITS - 1) / UNITS;
    // nx == 1 (small grids, one-XCD partitions, H264R_DB2_XCD=0): one counter, write-through
    // records, any wave on any XCD
#if !H264R_DB2_XCD
    nx = 1;
#endif
    unsigned xcc_reg = 0;
    if (nx > 1) asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_reg));
    const int xcc = (int)(xcc_reg & 15u) % nx;
    const int ngx = (ngroups - xcc + nx - 1) / nx;           // groups xcc, xcc + nx, ...
    int* counter = &sync[xcc];
    const bool local = nx > 1;                                // records: plain stores, kept in the XCD's L2
    const int items = ngx * (R1 - R0);
    for (;;) {
    __syncthreads();                                          // the previous item's LDS reads are done
    int tk = 0;
    if (threadIdx.x == 0) tk = atomicAdd(counter, 1);
    const int ticket = __builtin_amdgcn_readfirstlane(tk);
    if (ticket >= items) {
        xcd_drain_check(sync, sync + 8, nx, [&](int k) { return (ngroups - k + nx - 1) / nx * (R1 - R0); }, err);
        return;
    }
    const int ry = ticket / ngx, grp = (ticket - ry * ngx) * nx + xcc;
    // lane, opaque per item: what derives from it is recomputed per item, not hoisted out of
    // the ticket loop and kept live across it (that spilled 31 VGPRs)
    int lane = threadIdx.x;
    asm volatile("" : "+v"(lane));
    const int u = lane >> 2, q = lane & 3;
    const int y = R0 + ry;
    const int pic_raw = grp * UNITS + u;
    const bool active = pic_raw < b.num_pics;
    const int pic = active ? pic_raw : b.num_pics - 1;
    const bool above = y > R0, last_row = y == R1 - 1;
    // records live in two slots per picture (rows alternate); the tag names launch and row
    const uint32_t tag32 = (epoch << 12) | ((uint32_t)ry & 0xFFFu);
    const uint64_t tag_in = (uint64_t)((epoch << 12) | ((uint32_t)(ry - 1) & 0xFFFu)) << 32;   // rows alternate slots

    UnitLds& U = S[u];
    const size_t Wl = (size_t)g.W, Wc = (size_t)g.Wc;
    uint8_t* Y = b.out_y + (size_t)pic * g.ysz + (size_t)(y * 16) * Wl;               // MB row y
    uint8_t* Cb = b.out_u + (size_t)pic * g.csz + (size_t)(y * 8) * Wc;
    uint8_t* Cr = b.out_v + (size_t)pic * g.csz + (size_t)(y * 8) * Wc;
    const int p = q >> 1, d = q & 1;                                                    // my chroma plane / dword
    uint8_t* Cp = p ? Cr : Cb;
    const v4u* info_row = reinterpret_cast<const v4u*>(dbinfo + (size_t)pic * g.nmb + (size_t)y * W);
    // byte offsets of this unit's record rows in hb, through one wave-uniform descriptor
    const uint32_t hb_bytes = (uint32_t)b.num_pics * 2u * (uint32_t)W * RECG * 8u;
    const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc(hb, 0, hb_bytes, 0x00020000);
    const uint32_t rec_out = (uint32_t)(((size_t)pic * 2 + (ry & 1)) * W * RECG * 8);
    const uint32_t rec_in = (uint32_t)(((size_t)pic * 2 + ((ry + 1) & 1)) * W * RECG * 8);
    // pair k (granules 2k, 2k+1) of consumer lane c of MB m.  An MB's 12 pairs form three
    // 64-byte blocks, each stored by ONE instruction of the unit's four lanes (one whole
    // write-through segment instead of four partial ones): block 0 = the early pairs
    // (0,0) (0,1) (0,2) (1,0), block 1 = the early (2,0) (2,1) (2,2) (1,1), block 2 = the
    // late (1,2) (3,0) (3,1) (3,2).
    // blk * 4 + slot of pair k of lane c, nibble 3c + k of PAIR_POS (a select chain on the lane's
    // c compiled to a branch tree at every use)
    constexpr uint64_t PAIR_POS = 0xba9654873210ull;
    auto pair_off = [&](uint32_t base, int m, int c, int k) -> uint32_t {
        const uint32_t bs = (uint32_t)(PAIR_POS >> (4 * (c * 3 + k))) & 15u;
        return base + (uint32_t)(m * RECG) * 8u + bs * 16u;
    };
    auto load_pair = [&](int m, int k) -> v4u {
        return __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(hrs, pair_off(rec_in, m, q, k), 0, AUX_SC1));
    };

    // ---- window fetch: MBs m, m+1 -- 768 contiguous bytes of the MB-tiled reconstruction
    // (device_common.h), 16 bytes per load: luma rows 2i + p of MB m + d, and the chroma
    // chunk k = 4i + q (MB m + k / 8, plane (k / 4) & 1, rows 2 (k & 3) and 2 (k & 3) + 1)
    const uint8_t* rrow = recon + ((size_t)pic * g.nmb + (size_t)y * W) * RECON_MB;
    v4u wl[8], wc[4];
    auto fetch = [&](int m) {
        const uint8_t* ma = rrow + (size_t)min(m + d, W - 1) * RECON_MB;
#pragma unroll
        for (int i = 0; i < 8; ++i) wl[i] = load_global<v4u>(ma + (2 * i + p) * 16);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = 4 * i + q;
            wc[i] = load_global<v4u>(rrow + (size_t)min(m + (k >> 3), W - 1) * RECON_MB + RECON_CB + (k & 7) * 16);
        }
    };
    auto fill = [&](int m) {                                                            // registers -> ring slots
        const int sa = m % 3, sb = (m + 1) % 3, s = d ? sb : sa;
#pragma unroll
        for (int i = 0; i < 8; ++i) *reinterpret_cast<v4u*>(&U.y[2 * i + p][4 * s]) = wl[i];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = 4 * i + q, sk = i < 2 ? sa : sb, pl = (k >> 2) & 1, r = 2 * (k & 3);
            *reinterpret_cast<v2u*>(&U.c[pl][r][2 * sk]) = wc[i].xy;
            *reinterpret_cast<v2u*>(&U.c[pl][r + 1][2 * sk]) = wc[i].zw;
        }
    };
    // the fetch registers read on the paths that do not fill (the last window, a failed
    // wait), so that no path reaches the loop head with their loads pending
    auto consume_window = [&]() {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("" ::"v"(wl[i]));
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(wc[i]));
    };
    // Stores are issued by every lane on every path (the same count whatever the lane or the
    // picture), so that the waitcnt pass can count the operations younger than a load it
    // waits for.  Rows the row below still changes (luma 13..15, chroma 7) become a second
    // store of row 12 / 6 with the same bytes; units past the batch end store exactly what
    // the unit of the picture they duplicate stores.
    const int ylast = last_row ? 15 : 12, clast = last_row ? 7 : 6;
    // final MBs m, m+1 (adjacent): luma rows as two 16-byte halves from a lane pair, chroma
    // rows as two 8-byte halves
    auto store_pair = [&](int m) {
        const int sa = m % 3, sb = (m + 1) % 3, s = d ? sb : sa;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int r = min(2 * i + p, ylast);
            *reinterpret_cast<v4u*>(Y + (size_t)r * Wl + (m + d) * 16) = *reinterpret_cast<const v4u*>(&U.y[r][4 * s]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int pr = 4 * i + q, r = min(pr & 7, clast);
            uint8_t* dst = (pr >> 3 ? Cr : Cb) + (size_t)r * Wc + m * 8;
            *reinterpret_cast<v2u*>(dst) = *reinterpret_cast<const v2u*>(&U.c[pr >> 3][r][2 * sa]);
            *reinterpret_cast<v2u*>(dst + 8) = *reinterpret_cast<const v2u*>(&U.c[pr >> 3][r][2 * sb]);
        }
    };
    // one final MB: my luma rows 4q..4q+3 and chroma rows 4(q&1)..+3 of plane p
    auto store_one = [&](int m) {
        const int s = m % 3;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = min(4 * q + i, ylast);
            *reinterpret_cast<v4u*>(Y + (size_t)r * Wl + m * 16) = *reinterpret_cast<const v4u*>(&U.y[r][4 * s]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = min(4 * d + i, clast);
            *reinterpret_cast<v2u*>(Cp + (size_t)r * Wc + m * 8) = *reinterpret_cast<const v2u*>(&U.c[p][r][2 * s]);
        }
    };
    // granule i of consumer lane c of MB m, from the ring: luma row 12+i dword c (i < 4),
    // chroma plane c/2 row 2+i dword c&1 (i = 4, 5)
    auto granule = [&](int m, int c, int i) -> uint32_t {
        const int s = m % 3;
        return i < 4 ? U.y[12 + i][4 * s + c] : U.c[c >> 1][2 + i][2 * s + (c & 1)];
    };
    // publish pair k of consumer lane c of MB m.  Pairs are final either after H(m) ("early":
    // lanes 0 and 2, lane 1's pairs 0-1) or only after V(m+1) ("late": lane 1's pair 2 with
    // chroma dword 1, lane 3's three with luma dword 3 / chroma dword 1).
    auto publish_pair = [&](int m, int c, int k, uint32_t t) {
        const v4u v = {granule(m, c, 2 * k), t, granule(m, c, 2 * k + 1), t};
        const auto w = __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v);
        if (local) __builtin_amdgcn_raw_buffer_store_b128(w, hrs, pair_off(rec_out, m, c, k), 0, 0);
        else __builtin_amdgcn_raw_buffer_store_b128(w, hrs, pair_off(rec_out, m, c, k), 0, AUX_SC1);
    };
    // early pairs: 8, block j slot q from lane q; late pairs: 4, block 2 slot q from lane q
    auto early_c = [&](int lq, int j) { return lq < 3 ? (j ? 2 : 0) : 1; };
    auto early_k = [&](int lq, int j) { return lq < 3 ? lq : j; };
    auto late_c = [&](int lq) { return lq == 0 ? 1 : 3; };
    auto late_k = [&](int lq) { return lq == 0 ? 2 : lq - 1; };
    // DbInfo of MB m: 5 pieces of 16 bytes, piece q and (every lane) piece 4
    v4u ninf[2];
    auto load_info = [&](int m) {
        const v4u* src = info_row + (size_t)min(m, W - 1) * 5;
        ninf[0] = src[q];
        ninf[1] = src[4];
    };
    auto put_info = [&]() {
        *reinterpret_cast<v4u*>(&U.info[4 * q]) = ninf[0];
        *reinterpret_cast<v4u*>(&U.info[16]) = ninf[1];
    };

    TRACE(const unsigned long long tr_start = __builtin_amdgcn_s_memrealtime(); unsigned long long tph[4] = {0, 0, 0, 0};
          unsigned long long tm = __builtin_amdgcn_s_memtime();)
    bool ok = true;
    fetch(0);
    load_info(0);
    fill(0);
    put_info();
    __syncthreads();
    // one step; ODD is x's parity, known at each call site, so that a window's fetch (even
    // step) and fill (odd step) sit in one loop iteration and no load is pending across
    // the back edge (the waitcnt pass then needs no conservative waits)
    auto step = [&](const int x, auto odd_tag) {
        constexpr bool ODD = decltype(odd_tag)::value;
        const int sc = x % 3, sl = (x + 2) % 3;
        // 1. the record of MB (x, y-1) (checked after the vertical edges)
        uint64_t rin[6];
        if (above) {
#pragma unroll
            for (int k = 0; k < 3; ++k) { const v4u v = load_pair(x, k); rin[2 * k] = v.x | (uint64_t)v.y << 32; rin[2 * k + 1] = v.z | (uint64_t)v.w << 32; }
        }
        load_info(x + 1);                        // (clamped) younger than the record loads: not waited for there
        uint32_t inf[20];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const v4u v = *reinterpret_cast<const v4u*>(&U.info[4 * k]);
            inf[4 * k] = v.x; inf[4 * k + 1] = v.y; inf[4 * k + 2] = v.z; inf[4 * k + 3] = v.w;
        }
        // edge words of my chroma plane (par[3 + 3p ..], selected without indexing by p)
        const uint32_t cpar[3] = {p ? inf[14] : inf[11], p ? inf[15] : inf[12], p ? inf[16] : inf[13]};

        // 2. vertical edges of MB x (deblock.cc:488-504)
        uint32_t lcv[2];                         // chroma: left dwords of rows 4d+2+i after V(x)
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
                for (int k = 0; k < 4; ++k) pack4(c[4 + 4 * k], c[5 + 4 * k], c[6 + 4 * k], c[7 + 4 * k], a[k], bb[k]);
                U.y[ra][4 * sl + 3] = la;
                U.y[rb][4 * sl + 3] = lb;
                *reinterpret_cast<v4u*>(&U.y[ra][4 * sc]) = (v4u){a[0], a[1], a[2], a[3]};
                *reinterpret_cast<v4u*>(&U.y[rb][4 * sc]) = (v4u){bb[0], bb[1], bb[2], bb[3]};
            }
            // chroma plane p rows (4d + i, +2); chroma edge 0 = luma edge 0, edge 1 (col 4) =
            // luma edge 2; row j takes the bS of luma row 2j: segment j / 2 (deblock.cc:430-433, 460)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int ra = 4 * d + i, rb = ra + 2;
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
                lcv[i] = lb;                     // chroma rows 6 + i (lanes with d = 1)
            }
        }
        TRACE({ const unsigned long long t2 = __builtin_amdgcn_s_memtime(); tph[0] += t2 - tm; tm = t2; })
        // 3. what the next step needs, behind the record loads in issue order
        if (!ODD) fetch(min(x + 2, W - 1));                                             // next window

        // 4. the record of MB (x, y-1) from the row above: wait for this launch
        if (above) {
            auto ready = [&]() {
                bool r = true;
#pragma unroll
                for (int i = 0; i < 6; ++i) r &= (rin[i] & 0xFFFFFFFF00000000ull) == tag_in;
                return __builtin_amdgcn_readfirstlane(__all(r || !active)) != 0;   // wave-uniform
            };
            // the first check stands outside the re-poll loop, so that its wait covers the
            // record loads only (the loads issued after them stay in flight)
            if (!ready()) {
                WaitClock wc;
                do {
                    __builtin_amdgcn_s_sleep(1);
#pragma unroll
                    for (int k = 0; k < 3; ++k) { const v4u v = load_pair(x, k); rin[2 * k] = v.x | (uint64_t)v.y << 32; rin[2 * k + 1] = v.z | (uint64_t)v.w << 32; }
                    if (wait_give_up(err, wc)) {                 // bounded (device_common.h)
                        ok = false;
                        consume_window();
                        return;
                    }
                } while (!ready());
            }
        }
        // a band that starts below row 0 must not be filtered across its top edge (idc 1, or a
        // slice edge with idc 2): its top-edge strengths (bs[16..19] = info dword 4) are 0
        if (y == R0 && R0 > 0 && __builtin_amdgcn_readfirstlane(__any(active && inf[4] != 0)))
            __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        TRACE({ const unsigned long long t2 = __builtin_amdgcn_s_memtime(); tph[1] += t2 - tm; tm = t2; })
        // the late pairs of MB x-1 (luma dword 3, chroma dword 1), final after V(x): one per
        // lane.  At x = 0 the same store carries tag 0 -- never taken for ready -- onto MB 0's
        // pair, which step 1 overwrites.
        publish_pair(max(x - 1, 0), late_c(q), late_k(q), x ? tag32 : 0u);

        // 5. horizontal edges of MB x (deblock.cc:506-535)
        uint32_t wy[20], wcv[10];
        {
            // luma columns 4q .. 4q+3 (dword q), rows -4..15 (rows -4..-1: the record), pairs (j, j+2)
#pragma unroll
            for (int r = 0; r < 4; ++r) wy[r] = (uint32_t)rin[r];
#pragma unroll
            for (int r = 0; r < 16; ++r) wy[4 + r] = U.y[r][4 * sc + q];
            EdgeP eh[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) eh[e] = edge_params(inf[8 + (e == 0 ? 1 : 2)], bs_pair(inf[4 + e], q, q));
            s2 c[2][20];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int r = 0; r < 20; ++r) c[j][r] = unpack_cols(wy[r], j);
                filter2<true, false>(c[j][0], c[j][1], c[j][2], c[j][3], c[j][4], c[j][5], c[j][6], c[j][7], eh[0]);
#pragma unroll
                for (int e = 1; e < 4; ++e)
                    filter2<false, false>(c[j][4 * e], c[j][4 * e + 1], c[j][4 * e + 2], c[j][4 * e + 3], c[j][4 * e + 4],
                                          c[j][4 * e + 5], c[j][4 * e + 6], c[j][4 * e + 7], eh[e]);
            }
#pragma unroll
            for (int r = 1; r < 20; ++r) wy[r] = pack_cols(c[0][r], c[1][r]);
#pragma unroll
            for (int r = 0; r < 16; ++r) U.y[r][4 * sc + q] = wy[4 + r];
        }
        {
            // chroma plane p, columns 4d .. 4d+3 (dword d), rows -2..7; the halves of a pair sit
            // in segments 2d and 2d+1 of luma H edge 0 / 2
#pragma unroll
            for (int r = 0; r < 2; ++r) wcv[r] = (uint32_t)rin[4 + r];
#pragma unroll
            for (int r = 0; r < 8; ++r) wcv[2 + r] = U.c[p][r][2 * sc + d];
            EdgeP eh[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) eh[e] = edge_params(cpar[e == 0 ? 1 : 2], bs_pair(inf[4 + 2 * e], 2 * d, 2 * d + 1));
            s2 c[2][10];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int r = 0; r < 10; ++r) c[j][r] = unpack_cols(wcv[r], j);
                s2 d0 = c[j][0], d1 = c[j][9];
                filter2<true, true>(d0, d0, c[j][0], c[j][1], c[j][2], c[j][3], d1, d1, eh[0]);
                filter2<false, true>(d0, d0, c[j][4], c[j][5], c[j][6], c[j][7], d1, d1, eh[1]);
            }
#pragma unroll
            for (int r = 1; r < 10; ++r) wcv[r] = pack_cols(c[0][r], c[1][r]);
#pragma unroll
            for (int r = 0; r < 8; ++r) U.c[p][r][2 * sc + d] = wcv[2 + r];
        }
        TRACE({ const unsigned long long t2 = __builtin_amdgcn_s_memtime(); tph[2] += t2 - tm; tm = t2; })

        // 6. publish / store what is final now: the 16 granules of MB x that MB x+1 cannot
        // change, four per lane (at the row end the late ones are final too)
#pragma unroll
        for (int j = 0; j < 2; ++j) publish_pair(x, early_c(q, j), early_k(q, j), tag32);
        if (x == W - 1) publish_pair(x, late_c(q), late_k(q), tag32);
        if (above) {
            // rows 13..15 of MB (x, y-1), my luma dword; chroma row 7 of my plane, my dword
#pragma unroll
            for (int r = 1; r < 4; ++r) *reinterpret_cast<uint32_t*>(Y - (size_t)(4 - r) * Wl + x * 16 + 4 * q) = wy[r];
            *reinterpret_cast<uint32_t*>(Cp - Wc + x * 8 + 4 * d) = wcv[1];
        }
        __syncthreads();
        if (ODD) {
            if (x + 1 < W) {
                // window switch: MBs x-2, x-1 are final and leave the ring; x+1, x+2 come in
                store_pair(max(x - 2, 0));           // (x = 1: MB 1 again at x = 3)
                __syncthreads();                     // every lane has read the slots fill() reuses
                fill(x + 1);
            } else {
                consume_window();
            }
        }
        put_info();                                  // (stale after the last MB: never read)
        __syncthreads();
        TRACE({ const unsigned long long t2 = __builtin_amdgcn_s_memtime(); tph[3] += t2 - tm; tm = t2; })
    };
    // the back edge follows an odd step only: no path reaches the loop head with a load
    // of the even step pending
    for (int x = 0;; x += 2) {
        step(x, std::false_type());
        if (!ok || x + 1 >= W) break;
        step(x + 1, std::true_type());
        if (!ok || x + 2 >= W) break;
    }
    if (ok) {
        // the row end: the MBs the last window switch left in the ring (W-3 .. W-1 for even
        // W, W-2 .. W-1 for odd W)
        const int m0 = max(W - ((W & 1) ? 2 : 3), 0);
        if (W - m0 == 3) { store_pair(m0); store_one(m0 + 2); }
        else if (W - m0 == 2) store_pair(m0);
        else store_one(m0);
    } else if (!last_row) {                          // release the row below (the error is flagged)
        for (int x = 0; x < W; ++x)
            for (int k = 0; k < 3; ++k) {
                const v4u v = {0u, tag32, 0u, tag32};
                const auto w = __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v);
                if (local) __builtin_amdgcn_raw_buffer_store_b128(w, hrs, pair_off(rec_out, x, q, k), 0, 0);
                else __builtin_amdgcn_raw_buffer_store_b128(w, hrs, pair_off(rec_out, x, q, k), 0, AUX_SC1);
            }
    }
    // (indexed row-major over (row, group) whatever the XCD-local ticket numbering)
    TRACE(const int tix = ry * ngroups + grp;
          if (lane == 0 && tix < (1 << 16)) {
        h264r_db2_trace[tix][0] = tr_start; h264r_db2_trace[tix][1] = __builtin_amdgcn_s_memrealtime();
        for (int i = 0; i < 4; ++i) h264r_db2_trace[tix][2 + i] = tph[i];
        h264r_db2_trace[tix][6] = (unsigned long long)W; })
    }
}
