// k_deblock2.hip -- the in-loop deblocking filter for large batches: bands of MB rows
// walked in lock step, 8 lanes per (picture, MB row), packed 16-bit filters, LDS rings,
// output staged in LDS and stored as whole 64-byte row pieces.
//
// The reference filters MB by MB in raster order, vertical edges then horizontal edges
// (Deblock::deblock_pic, deblock.cc:537-552): along a row MB x needs MB x-1 finished,
// and MB (x, y) needs the samples MB (x+1, y-1)'s left edge wrote.  k_deblock
// (k_deblock.hip) spreads one MB over 32 lanes; its steps are short but latency-bound.
// Here the parallelism comes from the pictures of the batch: a 64-lane wave owns a BAND
// of H264R_DB2_BAND consecutive MB rows of 64 / (LPU * BAND) pictures, LPU =
// H264R_DB2_LPU lanes per (picture, row) "unit" (8; 4 is kept for A/B), and walks them
// in lock step, row rb of the band one MB behind row rb-1 (the least lag the reference's
// order allows: within one step every unit runs its vertical edges before any runs its
// horizontal edges, so MB x of the upper row has had MB x+1's left edge filtered when
// the lower row filters its top edge).
//
// A unit's lanes are (q, h), q = 0..3 the quarter of the MB, h = 0..LPU/4-1 the half of it:
//   vertical edges   lane q filters luma rows 4q .. 4q+3 as the pairs (r, r+2) and
//                    chroma plane q/2, rows 4(q&1) .. +3 -- filter_vertical deblock.cc:488-504;
//                    at 8 lanes lane h takes pair h of the two
//   horizontal edges lane q filters luma columns 4q .. 4q+3 as the pairs (c, c+2) and
//                    chroma plane q/2, columns 4(q&1) .. +3 -- filter_horizontal :506-535;
//                    at 8 lanes lane h takes pair h and the partner lane's result comes
//                    back by one DPP move to rebuild the dword
//
// Every operand is an s16x2 of two lines (mb_deblock2.h); the transposition between
// the two passes is free, since both read the MB from LDS.  Each unit's MB row lives
// in LDS as two MB slots (MB x in slot x & 1: the left neighbour and the current MB).
// Between a step's vertical and horizontal edges MB x-1 (final once MB x's left edge is
// filtered) is copied into the unit's output staging and MB x+1, fetched into registers
// during the previous step, takes its slot; the step ends by fetching MB x+2.
//
// Output staging (StageLds): the final samples are collected per group of 4 MBs, and a
// completed group is stored as one 64-byte piece per luma row and 32-byte pieces per chroma
// row.  Storing each MB's 16-byte row pieces as they became final had left the 128-byte
// lines in L2 partly written for 8 steps, so they were written back piecemeal: 2.8x the
// output bytes, 1.4-1.8 ms of the kernel (profiles/r05_l_deblock_store_ab.txt).  A unit
// with two slots, its staging and its share of the band-first row's UpLds takes 20.2 KiB
// per wave: 8 waves per CU (profiles/r05_aa_deblock_staging_ab.txt).
//
// Inside the band the row below reads MB x's bottom rows straight from the upper unit's
// ring slot (the upper row is on MB x+1 then: MB x is its left neighbour).  Only the
// band's bottom row hands its bottom rows to the next band (a wave of a later ticket):
// 24 naturally aligned 8-byte granules {data dword, tag} per MB, laid out so that lane q
// of the consuming row polls exactly the six it filters with (luma dword q of rows
// 12..15, chroma plane q/2 dword q&1 of rows 6..7) and the producing lanes publish
// exactly the six they hold after the horizontal pass.  Luma dword 3 and chroma dword 1
// change again with MB x+1's vertical edges and are published after them.  `sc1`
// polling loads until every granule carries this launch's tag (MI355X_MICROARCH.md R2
// granule hand-off).  Waves take tickets band-major, so a wave only waits on tickets
// taken earlier by running waves; every spin is bounded and flags the error word.
//
// Rows start and end one step apart, so at a given step some units are before their
// row's first MB or past its last: their filters run with bS 0 (no change) and their
// stores and publishes go to an out-of-range buffer offset (dropped by the buffer unit).
// Every memory operation is issued by every lane on every path, so the waitcnt pass can
// count the operations younger than a load it waits for.
//
// The split walk (launches of few pictures, h264r_host.hip): the same source built per plane,
// H264R_DB2_PL = 0 (k_deblock2y, luma) and 1 (k_deblock2c, chroma) -- the planes filter
// independently, so each plane's walk runs as its own waves beside the other's, each with only
// its plane's LDS arrays and hand-off pairs (luma pairs 0-1, chroma pair 2) and a shorter step.
//
// Sample ownership (each sample stored once, when final): a row stages MB x's rows
// 0..12 (chroma 0..6) once MB x+1's vertical edges are done, and the rows 13..15
// (chroma 7) of MB (x, y-1) after filtering its own top edge (into the upper unit's
// staging inside the band, into UpLds for the band's first row).  The launch's last row
// stages its own bottom rows.
#include "launch_cfg.h"
#include "mb_deblock.h"
#include "mb_deblock2.h"

using namespace h264r;

namespace {

constexpr int LPU = H264R_DB2_LPU;     // lanes per (picture, MB row) unit: 4 or 8
static_assert(LPU == 4 || LPU == 8, "H264R_DB2_LPU");
constexpr int UNITS = DEBLOCK2_UNITS;  // (picture, MB row) units per wave
constexpr int NH = LPU / 4;            // lanes per quad index q (8 lanes: the pairs of a dword split in two)
constexpr int BAND = H264R_DB2_BAND;   // MB rows per wave
#ifndef H264R_DB2_PL
#define H264R_DB2_PL 2                 // planes a wave filters: 2 both; 0 luma, 1 chroma (the split walk, Makefile)
#endif
constexpr int PL = H264R_DB2_PL;
constexpr bool DOY = PL != 1, DOC = PL != 0;
static_assert(PL == 2 || LPU == 8, "the split walk is built at 8 lanes per unit");
constexpr int PICS = UNITS / BAND;     // pictures per wave
#ifndef H264R_DB2_SG
#define H264R_DB2_SG 4                 // MBs per output-staging group (StageLds): 4 or 2
#endif
constexpr int SG = H264R_DB2_SG;
static_assert(SG == 4 || SG == 2, "H264R_DB2_SG");
static_assert(UNITS % BAND == 0, "a band divides the wave's units");
constexpr int RECG = 24;               // granules per MB record: [consumer lane c 0..3][i 0..5]
constexpr int AUX_SC1 = 16;            // buffer-op cache policy: sc1 (write-through store, L2-served load)
constexpr int RSRC_W3 = 0x00020000;    // buffer descriptor word 3 (gfx9 raw buffer, range-checked)
constexpr uint32_t OOB = 0x80000000u;  // added to an offset: past every range (loads 0, stores dropped)

// One unit's MB row in LDS: two MB slots and the DbInfo -- 848 B.  The unit stride of 212
// dwords puts consecutive units 20 banks apart (mod 32).
// (the split walk's builds keep their plane's arrays only: every layout's unit stride stays
// 20 banks mod 32)
constexpr int YR = DOY ? 16 : 0, CR = DOC ? 8 : 0;   // luma / chroma rows held
struct alignas(16) UnitLds {
    uint32_t y[YR][8];        // luma rows 0..15; MB x in slot s = x & 1: dwords 4s .. 4s+3
    uint32_t c[2][CR][4];     // chroma plane, rows 0..7; slot s = dwords 2s, 2s+1
    uint32_t info[20];        // DbInfo of the MB being filtered (zeros: no MB this step)
};
static_assert(sizeof(UnitLds) == (PL == 2 ? 848 : PL == 0 ? 592 : 336), "UnitLds layout");

// A unit's output staging: the final samples of its MB row, collected per group of 4 MBs, so
// that the output planes take whole 64-byte pieces of their luma rows and 32-byte pieces of their
// chroma rows (16- and 8-byte row pieces, each of a line the walk completes only 8 steps later,
// had left L2 partly written: 2.8x the output bytes written, and the stores took 1.8 of the
// kernel's 5.0 ms; profiles/r05_l_deblock_store_ab.txt).  Rows 13..15 (chroma 7) of a row are
// final only after the row below has filtered its top edges: the unit below writes them into
// this unit's staging (same wave), or, for the band's first row, into the UpLds of its picture
// (the row above is another wave's).  1.5 KiB per unit: 8 waves per CU at 8 lanes per unit.
// (SG = 2: 2-MB groups, 32-byte luma / 16-byte chroma row pieces, 784 B per unit with a unit
// stride 4 banks apart -- 13.0 KiB per wave, 12 waves per CU)
struct alignas(16) StageLds {
    uint32_t y[YR][SG][4];     // luma rows 0..15, MB m % SG of the group: 16 bytes
    uint32_t c[2][CR][SG][2];  // chroma plane, rows 0..7, MB m % SG: 8 bytes
    uint32_t pad[SG == 4 ? 20 : 4];   // unit stride 404 (SG 4) / 196 (SG 2) dwords: 20 / 4 banks apart
};
static_assert(SG != 4 || sizeof(StageLds) == (PL == 2 ? 1616 : PL == 0 ? 1104 : 592), "StageLds layout");
struct alignas(16) UpLds {     // the band's first row: rows 13..15 (chroma 7) of the row above
    uint32_t yu[DOY ? 3 : 0][SG][4];
    uint32_t cu[2][DOC ? SG : 0][2];
};

typedef uint32_t v4u __attribute__((ext_vector_type(4)));   // native vectors: registers, not stack
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

// {byte j, byte j + 2} of one dword as an s16x2 (the column pair (j, j+2)).
DEV s2 unpack_cols(uint32_t w, int j) { return as_s2(__builtin_amdgcn_perm(w, w, 0x0C000C00u | ((uint32_t)(j + 2) << 16) | (uint32_t)j)); }
// Column pairs (0, 2) and (1, 3) back into one dword.
DEV uint32_t pack_cols(s2 c0, s2 c1) { return __builtin_amdgcn_perm(as_w(c1), as_w(c0), 0x06020400u); }
DEV s2 bs_pair(uint32_t w, int slo, int shi) { return (s2){(short)((w >> (8 * slo)) & 255), (short)((w >> (8 * shi)) & 255)}; }

template <int AUX = 0>
DEV void st16(__amdgpu_buffer_rsrc_t r, uint32_t off, v4u v)
{
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v), r, off, 0, AUX);
}
template <int AUX = 0>
DEV void st8(__amdgpu_buffer_rsrc_t r, uint32_t off, v2u v)
{
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned int, v), r, off, 0, AUX);
}
template <int AUX = 0>
DEV void st4(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t v) { __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, AUX); }
#ifndef H264R_DB2_OUT_AUX
#define H264R_DB2_OUT_AUX 0                // cache policy of the output-plane stores (measurement knob)
#endif
constexpr int OUT_AUX = H264R_DB2_OUT_AUX;

}  // namespace

#ifndef H264R_DB2_KERNEL
#define H264R_DB2_KERNEL k_deblock2        // the split walk's builds are k_deblock2y / k_deblock2c (Makefile)
#endif
#ifdef H264R_TRACE
// Timing trace (trace builds only: make EXTRA=-DH264R_TRACE): per ticket {start, end
// (s_memrealtime, 100 MHz), then s_memtime cycles spent in: V pass, record wait, output
// stores + staging + fill, H pass + publishes + next fetch}.
#if H264R_DB2_PL == 0
#define h264r_db2_trace h264r_db2y_trace
#define h264r_db2_trace_copy h264r_db2y_trace_copy
#elif H264R_DB2_PL == 1
#define h264r_db2_trace h264r_db2c_trace
#define h264r_db2_trace_copy h264r_db2c_trace_copy
#endif
__device__ unsigned long long h264r_db2_trace[1 << 16][8];
#define TRACE(...) __VA_ARGS__
extern "C" void h264r_db2_trace_copy(void* dst) { (void)hipMemcpyFromSymbol(dst, HIP_SYMBOL(h264r_db2_trace), sizeof(h264r_db2_trace)); }
#else
#define TRACE(...)
#endif

// hb: records [pic][band & 1][W][RECG] granules {dword, tag}, moved as 16-byte pairs (two
// granules; each 8-byte half observed untorn on gfx950, MI355X_MICROARCH.md visibility:
// the tag check stays per granule); sync[0..nx): ticket counters; epoch < 2^20 (the host
// restarts from zeroed records before it wraps).
// XCD-local hand-off (H264R_DB2_XCD, default): the bands of a picture group all run on
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
#ifndef H264R_DB2_DIAG
#define H264R_DB2_DIAG 0   // diagnostic builds only (wrong output): bit 0 drops the output stores, bit 1 fetches MB 0
#endif
// Register budget: the waves a CU holds are set by LDS (UnitLds + StageLds per unit + UpLds per
// picture: 20.2 KiB, 8 waves per CU at 8 lanes per unit); asking for 2 waves per SIMD keeps the
// compiler from parking values in AGPRs (at a 512-register budget it did, and the wave's VGPR +
// AGPR footprint of 257 left one wave per SIMD)
#define H264R_DB2_WAVES_PER_EU (H264R_DB2_PL == 1 ? 4 : H264R_DB2_PL == 0 ? 3 : H264R_DB2_LPU == 8 ? (H264R_DB2_SG == 2 ? 3 : 2) : 1)   // split builds: 3 / 4
extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(H264R_DB2_WAVES_PER_EU, H264R_DB2_WAVES_PER_EU))) void H264R_DB2_KERNEL(
    h264r_batch b, const DbInfo* __restrict__ dbinfo, uint64_t* hb, int* sync, int* err, uint32_t epoch, int2 rows, int nx,
    const uint8_t* __restrict__ recon)
{
    __shared__ UnitLds S[UNITS];
    __shared__ StageLds G[UNITS];
    __shared__ UpLds UP[PICS];
#ifdef H264R_DB2_LDS_PAD
    // measurement builds only: LDS padding that lowers the resident waves per CU
    __shared__ uint32_t lds_pad[H264R_DB2_LDS_PAD / 4];
    if (threadIdx.x == 0 && epoch == 0xFFFFFFFFu) { lds_pad[0] = 1; __syncthreads(); err[0] = lds_pad[0]; }
#endif
    const Geom g = make_geom(b.width_mbs, b.height_mbs);
    const int W = g.wmb, R0 = rows.x, R1 = rows.y;
    const int ngroups = (b.num_pics + PICS - 1) / PICS;
    const int nbands = (R1 - R0 + BAND - 1) / BAND;
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
    const int items = ngx * nbands;
    for (;;) {
    __syncthreads();                                          // the previous item's LDS reads are done
    int tk = 0;
    if (threadIdx.x == 0) tk = atomicAdd(counter, 1);
    const int ticket = __builtin_amdgcn_readfirstlane(tk);
    if (ticket >= items) {
        xcd_drain_check(sync, sync + 8, nx, [&](int k) { return (ngroups - k + nx - 1) / nx * nbands; }, err);
        return;
    }
    const int band = ticket / ngx, grp = (ticket - band * ngx) * nx + xcc;
    // lane, opaque per item: what derives from it is recomputed per item, not hoisted out of
    // the ticket loop and kept live across it
    int lane = threadIdx.x;
    asm volatile("" : "+v"(lane));
    // unit u; q = the unit's quarter (luma rows / dword column 4q.., chroma plane q/2, dword q&1);
    // with 8 lanes per unit, h = which half of q's two row / column pairs this lane filters
    const int u = lane / LPU, q8 = lane % LPU, q = q8 / NH, h = q8 % NH;
    const int rb = u / PICS, pu = u - rb * PICS;              // row in the band, picture in the group
    const int y = R0 + band * BAND + rb;
    const int pic0 = grp * PICS, npg = min(PICS, b.num_pics - pic0);
    const bool active = pu < npg && y < R1;                  // units past the batch or the rows: no MB
    const int pic = pic0 + min(pu, npg - 1), yc = min(y, R1 - 1);
    const bool above = y > R0, last_row = y == R1 - 1;
    // records live in two slots per picture (bands alternate); the tag names launch and band
    const uint32_t tag32 = (epoch << 12) | ((uint32_t)band & 0xFFFu);
    const uint64_t tag_in = (uint64_t)((epoch << 12) | ((uint32_t)(band - 1) & 0xFFFu)) << 32;
    const bool polls = active && rb == 0 && above;            // the band above's records
    const bool publishes = active && rb == BAND - 1 && !last_row;

    UnitLds& U = S[u];
    const UnitLds& A = S[rb ? u - PICS : u];                  // the unit of the row above (rb > 0)
    StageLds& T = G[u];
    StageLds& TA = G[rb ? u - PICS : u];                      // its staging
    UpLds& TU = UP[pu];                                       // (rb == 0) the row above's final rows
    const uint32_t Wl = (uint32_t)g.W, Wc = (uint32_t)g.Wc;
    const uint32_t ysz = (uint32_t)g.ysz, csz = (uint32_t)g.csz;
    // the group's output planes through wave-uniform descriptors; per-lane byte offsets of
    // row 0 of MB row y (OOB for units without an MB)
    const __amdgpu_buffer_rsrc_t rY = __builtin_amdgcn_make_buffer_rsrc(b.out_y + (size_t)pic0 * g.ysz, 0, (int)(npg * ysz), RSRC_W3);
    const __amdgpu_buffer_rsrc_t rU = __builtin_amdgcn_make_buffer_rsrc(b.out_u + (size_t)pic0 * g.csz, 0, (int)(npg * csz), RSRC_W3);
    const __amdgpu_buffer_rsrc_t rV = __builtin_amdgcn_make_buffer_rsrc(b.out_v + (size_t)pic0 * g.csz, 0, (int)(npg * csz), RSRC_W3);
    const uint32_t yrow = active ? (uint32_t)(pic - pic0) * ysz + (uint32_t)y * 16u * Wl : OOB;
    const uint32_t crow = active ? (uint32_t)(pic - pic0) * csz + (uint32_t)y * 8u * Wc : OOB;
    const int p = q >> 1, d = q & 1;                                                    // my chroma plane / dword
    const v4u* info_row = reinterpret_cast<const v4u*>(dbinfo + (size_t)pic * g.nmb + (size_t)yc * W);
    // byte offsets of this unit's record rows in hb, through one wave-uniform descriptor
    const uint32_t hb_bytes = (uint32_t)b.num_pics * 2u * (uint32_t)W * RECG * 8u;
    const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc(hb, 0, (int)hb_bytes, RSRC_W3);
    const uint32_t rec_out = publishes ? (uint32_t)(((size_t)pic * 2 + (band & 1)) * W * RECG * 8) : OOB;
    const uint32_t rec_in = polls ? (uint32_t)(((size_t)pic * 2 + ((band + 1) & 1)) * W * RECG * 8) : OOB;
    // pair k (granules 2k, 2k+1) of consumer lane c of MB m.  An MB's 12 pairs form three
    // 64-byte blocks, each stored by ONE instruction of the unit's four lanes: block 0 =
    // the early pairs (0,0) (0,1) (0,2) (1,0), block 1 = the early (2,0) (2,1) (2,2) (1,1),
    // block 2 = the late (1,2) (3,0) (3,1) (3,2).  blk * 4 + slot of pair k of lane c is
    // nibble 3c + k of PAIR_POS.
    constexpr uint64_t PAIR_POS = 0xba9654873210ull;
    auto pair_off = [&](uint32_t base, int m, int c, int k) -> uint32_t {
        const uint32_t bs = (uint32_t)(PAIR_POS >> (4 * (c * 3 + k))) & 15u;
        return base + (uint32_t)(m * RECG) * 8u + bs * 16u;
    };

    // ---- one MB of the MB-tiled reconstruction (device_common.h), 16 bytes per load:
    // luma rows q8 + LPU i, chroma chunks q8 + LPU j (chunk k: plane k / 4, rows 2 (k & 3), +1)
    const uint8_t* rrow = recon + ((size_t)pic * g.nmb + (size_t)yc * W) * RECON_MB;
    constexpr int NLR = 16 / LPU, NCK = 8 / LPU;
    v4u wl[NLR], wc[NCK];
    auto fetch = [&](int m) {
#if H264R_DB2_DIAG & 2
        m = 0;                           // diagnostic build: every fetch reads MB 0 (L2-resident)
#endif
        const uint8_t* ma = rrow + (size_t)min(max(m, 0), W - 1) * RECON_MB;
        if constexpr (DOY) {
#pragma unroll
            for (int i = 0; i < NLR; ++i) wl[i] = load_global<v4u>(ma + (LPU * i + q8) * 16);
        }
        if constexpr (DOC) {
#pragma unroll
            for (int j = 0; j < NCK; ++j) wc[j] = load_global<v4u>(ma + RECON_CB + (LPU * j + q8) * 16);
        }
    };
    auto fill = [&](int s) {                                                            // registers -> ring slot s
        if constexpr (DOY) {
#pragma unroll
            for (int i = 0; i < NLR; ++i) *reinterpret_cast<v4u*>(&U.y[LPU * i + q8][4 * s]) = wl[i];
        }
#pragma unroll
        for (int j = 0; j < NCK; ++j) {
            const int k = LPU * j + q8, pl = k >> 2, r = 2 * (k & 3);
            if (DOC) {
                *reinterpret_cast<v2u*>(&U.c[pl][r][2 * s]) = wc[j].xy;
                *reinterpret_cast<v2u*>(&U.c[pl][r + 1][2 * s]) = wc[j].zw;
            }
        }
    };
    // Rows 0..12 (chroma 0..6) of a row are final once the next MB's left edge is filtered, rows
    // 13..15 (chroma 7) once the row below has filtered its top edges -- or at once in the
    // launch's last row, and never in this wave for the band's last row (the next band's first
    // row stores them).
    const int ylast = last_row || rb < BAND - 1 ? 15 : 12, clast = last_row || rb < BAND - 1 ? 7 : 6;
    // final MB m (slot s) into the staging: luma rows 4i + q; chroma instruction i: plane i / 2,
    // row 4 (i & 1) + q (rows 13..15 / 7 are overwritten by the row below when it has filtered them)
    auto stage_own = [&](int m, int s) {
        const int mc = max(m, 0);
        if constexpr (DOY) {
#pragma unroll
            for (int i = 0; i < NLR; ++i) {
                const int r = LPU * i + q8;
                *reinterpret_cast<v4u*>(&T.y[r][mc % SG][0]) = *reinterpret_cast<const v4u*>(&U.y[r][4 * s]);
            }
        }
        if constexpr (DOC) {
#pragma unroll
            for (int i = 0; i < NLR; ++i) {
                const int k = LPU * i + q8, pl = k >> 3, r = k & 7;
                *reinterpret_cast<v2u*>(&T.c[pl][r][mc % SG][0]) = *reinterpret_cast<const v2u*>(&U.c[pl][r][2 * s]);
            }
        }
    };
    // The groups that are complete at the end of a step, stored by the whole wave: each unit's
    // flag (its lanes agree) as a wave-uniform mask, per unit one luma instruction (16 rows x
    // 4 MBs = 64 lanes) and one chroma instruction per plane (8 rows x 4 MBs); a group cut by the
    // row end stores its MBs only.  Byte offsets per lane, OOB for lanes without a sample
    // (dropped by the buffer unit).
    auto store_groups = [&](int xs) {
        const int mo = xs - 1;                                   // final since V(xs), rows 13..15 now
        const bool own = active && mo >= 0 && mo < W;
        // lane = (row r, MB pp of the group); with SG = 2 lanes 32..63 have no row (r >= 16)
        const int r = lane / SG, pp = lane % SG, rr = min(r, 15), cp = rr >> 3, cr = rr & 7;
        for (uint64_t bm = __ballot(own && q8 == 0 && (mo % SG == SG - 1 || mo == W - 1)); bm; bm &= bm - 1) {
            const int l0 = __builtin_ctzll(bm), u2 = l0 / LPU;
            const int m2 = __builtin_amdgcn_readlane(mo, l0), yl2 = __builtin_amdgcn_readlane(ylast, l0);
            const int cl2 = __builtin_amdgcn_readlane(clast, l0);
            const uint32_t yr2 = (uint32_t)__builtin_amdgcn_readlane((int)yrow, l0);
            const uint32_t cr2 = (uint32_t)__builtin_amdgcn_readlane((int)crow, l0);
            const int g0 = m2 & ~(SG - 1);
            const bool inrow = g0 + pp <= m2 && r < 16;
            if constexpr (DOY)
                st16<OUT_AUX>(rY, r <= yl2 && inrow ? yr2 + (uint32_t)r * Wl + (uint32_t)(g0 + pp) * 16u : OOB,
                              *reinterpret_cast<const v4u*>(&G[u2].y[rr][pp][0]));
            if constexpr (DOC) {
                const uint32_t off = cr <= cl2 && inrow ? cr2 + (uint32_t)cr * Wc + (uint32_t)(g0 + pp) * 8u : OOB;
                const v2u cv = *reinterpret_cast<const v2u*>(&G[u2].c[cp][cr][pp][0]);
                st8<OUT_AUX>(rU, cp == 0 ? off : OOB, cv);
                st8<OUT_AUX>(rV, cp == 1 ? off : OOB, cv);
            }
        }
        // the band's first row: rows 13..15 (chroma 7) of the row above, final since H(xs)
        const bool up = active && rb == 0 && above && xs >= 0 && xs < W;
        for (uint64_t bm = __ballot(up && q8 == 0 && (xs % SG == SG - 1 || xs == W - 1)); bm; bm &= bm - 1) {
            const int l0 = __builtin_ctzll(bm), pu2 = l0 / LPU;     // rb == 0: unit = picture
            const int x2 = __builtin_amdgcn_readlane(xs, l0);
            const uint32_t yr2 = (uint32_t)__builtin_amdgcn_readlane((int)yrow, l0);
            const uint32_t cr2 = (uint32_t)__builtin_amdgcn_readlane((int)crow, l0);
            const int g0 = x2 & ~(SG - 1);
            const bool inrow = g0 + pp <= x2 && r < 16;
            if constexpr (DOY)
                st16<OUT_AUX>(rY, r < 3 && inrow ? yr2 - (uint32_t)(3 - r) * Wl + (uint32_t)(g0 + pp) * 16u : OOB,
                              *reinterpret_cast<const v4u*>(&UP[pu2].yu[min(r, 2)][pp][0]));
            if constexpr (DOC) {
                const uint32_t off = r < 2 && inrow ? cr2 - Wc + (uint32_t)(g0 + pp) * 8u : OOB;
                const v2u cv = *reinterpret_cast<const v2u*>(&UP[pu2].cu[r & 1][pp][0]);
                st8<OUT_AUX>(rU, r == 0 ? off : OOB, cv);
                st8<OUT_AUX>(rV, r == 1 ? off : OOB, cv);
            }
        }
    };
    // granule i of consumer lane c of MB m in slot s: luma row 12+i dword c (i < 4), chroma
    // plane c/2 row 2+i dword c&1 (i = 4, 5)
    auto granule = [&](int s, int c, int i) -> uint32_t {
        return i < 4 ? U.y[12 + i][4 * s + c] : U.c[c >> 1][2 + i][2 * s + (c & 1)];
    };
    // publish pair k of consumer lane c of MB m (slot s).  Pairs are final either after H(m)
    // ("early": lanes 0 and 2, lane 1's pairs 0-1) or only after V(m+1) ("late": lane 1's
    // pair 2 with chroma dword 1, lane 3's three with luma dword 3 / chroma dword 1).
    auto publish_pair = [&](uint32_t base, int m, int s, int c, int k) {
        const v4u v = {granule(s, c, 2 * k), tag32, granule(s, c, 2 * k + 1), tag32};
        if (local) st16(hrs, pair_off(base, m, c, k), v);
        else st16<AUX_SC1>(hrs, pair_off(base, m, c, k), v);
    };
    auto early_c = [&](int lq, int j) { return lq < 3 ? (j ? 2 : 0) : 1; };
    auto early_k = [&](int lq, int j) { return lq < 3 ? lq : j; };
    auto late_c = [&](int lq) { return lq == 0 ? 1 : 3; };
    auto late_k = [&](int lq) { return lq == 0 ? 2 : lq - 1; };
    // DbInfo of MB m: 5 pieces of 16 bytes; 4 lanes: piece q and (every lane) piece 4; 8 lanes:
    // piece min(q8, 4)
    constexpr int NINF = LPU == 4 ? 2 : 1;
    v4u ninf[NINF];
    auto load_info = [&](int m) {
        const v4u* src = info_row + (size_t)min(max(m, 0), W - 1) * 5;
        ninf[0] = src[min(q8, 4)];
        if (NINF == 2) ninf[NINF - 1] = src[4];
    };
    auto put_info = [&](bool ok) {      // zeros (bS 0: no edge filtered) when there is no MB
        const v4u z = {0u, 0u, 0u, 0u};
        *reinterpret_cast<v4u*>(&U.info[4 * min(q8, 4)]) = ok ? ninf[0] : z;
        if (NINF == 2) *reinterpret_cast<v4u*>(&U.info[16]) = ok ? ninf[NINF - 1] : z;
    };
    // a value of the lane holding the other half of this lane's pairs (8 lanes per unit)
    auto partner = [&](uint32_t v) -> uint32_t {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    };

    TRACE(const unsigned long long tr_start = __builtin_amdgcn_s_memrealtime(); unsigned long long tph[4] = {0, 0, 0, 0};
          unsigned long long tm = __builtin_amdgcn_s_memtime();)
    bool ok = true;
    // row rb filters MB x = s - rb at step s; steps -2 and -1 bring MBs 0 and 1 in, the last
    // step (x = W on the band's last row) stores MB W-1
    const int s0 = -2, s1 = W + BAND - 1;
    int x = s0 - rb;
    // the record of MB (m, y-1) from the band above, as {data, tag} granules (OOB: zeros)
    uint64_t rin[6];
    auto load_record = [&](int m) {
        const uint32_t base = active && m >= 0 && m < W ? rec_in : OOB;
#pragma unroll
        for (int k = PL == 1 ? 2 : 0; k < (PL == 0 ? 2 : 3); ++k) {       // luma pairs 0, 1; chroma pair 2
            const v4u v = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(hrs, pair_off(base, max(m, 0), q, k), 0, AUX_SC1));
            rin[2 * k] = v.x | (uint64_t)v.y << 32; rin[2 * k + 1] = v.z | (uint64_t)v.w << 32;
        }
    };
    put_info(false);                     // the first step has no MB
    wave_sync();
    // the loads every step ends with, in the same order, so that the loop head sees one state
    fetch(x + 1);
    load_info(x + 1);
    for (int s = s0; s <= s1; ++s, ++x) {
        const bool xok = active && x >= 0 && x < W;
        const int sl = (x + 1) & 1, sc = x & 1;          // slots of MBs x-1 and x
        // 1. this MB's DbInfo
        uint32_t inf[20];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const v4u v = *reinterpret_cast<const v4u*>(&U.info[4 * k]);
            inf[4 * k] = v.x; inf[4 * k + 1] = v.y; inf[4 * k + 2] = v.z; inf[4 * k + 3] = v.w;
        }
        // edge words of my chroma plane (par[3 + 3p ..], selected without indexing by p)
        const uint32_t cpar[3] = {p ? inf[14] : inf[11], p ? inf[15] : inf[12], p ? inf[16] : inf[13]};

        // 2. vertical edges of MB x (deblock.cc:488-504)
        {
          if constexpr (DOY) {
            // luma rows (4q + i, 4q + i + 2): bS of V edge e, segment q = byte 4e + q
            EdgeP ev[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) ev[e] = edge_params(inf[8 + (e == 0 ? 0 : 2)], bs_pair(inf[e], q, q));
#pragma unroll
            for (int ii = 0; ii < 2 / NH; ++ii) {
                const int i = NH == 2 ? h : ii;
                const int ra = 4 * q + i, rb2 = ra + 2;
                uint32_t la = U.y[ra][4 * sl + 3], lb = U.y[rb2][4 * sl + 3];
                const v4u Av = *reinterpret_cast<const v4u*>(&U.y[ra][4 * sc]);
                const v4u Bv = *reinterpret_cast<const v4u*>(&U.y[rb2][4 * sc]);
                uint32_t a[4] = {Av.x, Av.y, Av.z, Av.w}, bb[4] = {Bv.x, Bv.y, Bv.z, Bv.w};
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
                U.y[rb2][4 * sl + 3] = lb;
                *reinterpret_cast<v4u*>(&U.y[ra][4 * sc]) = (v4u){a[0], a[1], a[2], a[3]};
                *reinterpret_cast<v4u*>(&U.y[rb2][4 * sc]) = (v4u){bb[0], bb[1], bb[2], bb[3]};
            }
          }
            // the record of MB (x, y-1) from the band above, checked after the vertical edges
            // (issued here rather than at the step head: live across the luma pass its registers
            // spilled at three waves per SIMD)
            load_record(x);
            // chroma plane p rows (4d + i, +2); chroma edge 0 = luma edge 0, edge 1 (col 4) =
            // luma edge 2; row j takes the bS of luma row 2j: segment j / 2 (deblock.cc:430-433, 460)
          if constexpr (DOC) {
#pragma unroll
            for (int ii = 0; ii < 2 / NH; ++ii) {
                const int i = NH == 2 ? h : ii;
                const int ra = 4 * d + i, rb2 = ra + 2;
                EdgeP ec[2];
#pragma unroll
                for (int e = 0; e < 2; ++e)
                    ec[e] = edge_params(cpar[e == 0 ? 0 : 2], bs_pair(inf[2 * e], ra >> 1, rb2 >> 1));
                uint32_t la = U.c[p][ra][2 * sl + 1], lb = U.c[p][rb2][2 * sl + 1];
                const v2u Av = *reinterpret_cast<const v2u*>(&U.c[p][ra][2 * sc]);
                const v2u Bv = *reinterpret_cast<const v2u*>(&U.c[p][rb2][2 * sc]);
                uint32_t a[2] = {Av.x, Av.y}, bb[2] = {Bv.x, Bv.y};
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
                U.c[p][rb2][2 * sl + 1] = lb;
                *reinterpret_cast<v2u*>(&U.c[p][ra][2 * sc]) = (v2u){a[0], a[1]};
                *reinterpret_cast<v2u*>(&U.c[p][rb2][2 * sc]) = (v2u){bb[0], bb[1]};
            }
          }
        }
        TRACE({ const unsigned long long t2 = __builtin_amdgcn_s_memtime(); tph[0] += t2 - tm; tm = t2; })

        // 4. the record of MB (x, y-1) from the band above: wait for this launch
        auto ready = [&]() {
            bool r = true;
#pragma unroll
            for (int i = PL == 1 ? 4 : 0; i < (PL == 0 ? 4 : 6); ++i) r &= (rin[i] & 0xFFFFFFFF00000000ull) == tag_in;
            return __builtin_amdgcn_readfirstlane(__all(r || !(polls && xok))) != 0;   // wave-uniform
        };
        if (!ready()) {
            // every reload is checked before any exit of the loop, so that no path leaves it
            // with a load pending (the waitcnt pass would otherwise drain at the step head)
            WaitClock wclk;
            bool give_up = false;
            for (;;) {
                __builtin_amdgcn_s_sleep(1);
                load_record(x);
                if (ready()) break;
                if (wait_give_up(err, wclk)) { give_up = true; break; }   // bounded (device_common.h)
            }
            if (give_up) { ok = false; break; }
        }
        // a launch that starts below row 0 must not be filtered across its top edge (idc 1, or a
        // slice edge with idc 2): its top-edge strengths (bs[16..19] = info dword 4) are 0
        if (R0 > 0 && band == 0 && __builtin_amdgcn_readfirstlane(__any(rb == 0 && xok && inf[4] != 0)))
            __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        wave_sync();                             // V(x) of every unit is in LDS
        TRACE({ const unsigned long long t2 = __builtin_amdgcn_s_memtime(); tph[1] += t2 - tm; tm = t2; })
        // the late pairs of MB x-1 (luma dword 3, chroma dword 1), final after V(x) (at x = W:
        // after H(W-1)): one per lane
        if constexpr (PL == 2)
            publish_pair(active && x >= 1 && x <= W && h == 0 ? rec_out : OOB, max(x - 1, 0), sl, late_c(q), late_k(q));
        else if constexpr (PL == 0)      // luma dword 3: lanes (3, h) publish pair h
            publish_pair(active && x >= 1 && x <= W && q == 3 ? rec_out : OOB, max(x - 1, 0), sl, 3, h);
        else                             // chroma dword 1 (consumers 1, 3): lanes (q odd, 0)
            publish_pair(active && x >= 1 && x <= W && h == 0 && (q & 1) ? rec_out : OOB, max(x - 1, 0), sl, q, 2);
        // rows -4..-1 (chroma -2..-1) of MB x's top edge for rows 1.. of the band: the upper unit's
        // left slot (the upper row is on MB x+1), read before that slot is refilled below
        if (rb) {
            if constexpr (DOY) {
#pragma unroll
                for (int r = 0; r < 4; ++r) rin[r] = A.y[12 + r][4 * sc + q];
            }
            if constexpr (DOC) {
#pragma unroll
                for (int r = 0; r < 2; ++r) rin[4 + r] = A.c[p][6 + r][2 * sc + d];
            }
        }
        // 5. MB x-1 is final (V(x) done): it leaves the ring, and MB x+1 (fetched during the
        // previous step) takes its slot with its DbInfo
#if !(H264R_DB2_DIAG & 1)
        // the groups the previous step completed (issued here, a whole step before the next wait
        // on this wave's loads, which vmcnt orders behind them), read before MB x-1 takes the
        // first slot of the next group (a wave's LDS operations execute in issue order)
        store_groups(x - 1);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#endif
        stage_own(x - 1, sl);                    // MB x-1 is final (rows 13..15: below)
        wave_sync();                             // every lane has read slot sl
        fill(sl);
        put_info(active && x + 1 >= 0 && x + 1 < W);
        TRACE({ const unsigned long long t2 = __builtin_amdgcn_s_memtime(); tph[2] += t2 - tm; tm = t2; })

        // 6. horizontal edges of MB x (deblock.cc:506-535); rows -4..-1 from the record
        uint32_t wy[20], wcv[10];
        {
        if constexpr (DOY) {
#pragma unroll
            for (int r = 0; r < 4; ++r) wy[r] = (uint32_t)rin[r];
#pragma unroll
            for (int r = 0; r < 16; ++r) wy[4 + r] = U.y[r][4 * sc + q];
            EdgeP eh[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) eh[e] = edge_params(inf[8 + (e == 0 ? 1 : 2)], bs_pair(inf[4 + e], q, q));
            s2 c[2 / NH][20];
#pragma unroll
            for (int jj = 0; jj < 2 / NH; ++jj) {
                const int j = NH == 2 ? h : jj;
#pragma unroll
                for (int r = 0; r < 20; ++r) c[jj][r] = unpack_cols(wy[r], j);
                filter2<true, false>(c[jj][0], c[jj][1], c[jj][2], c[jj][3], c[jj][4], c[jj][5], c[jj][6], c[jj][7], eh[0]);
#pragma unroll
                for (int e = 1; e < 4; ++e)
                    filter2<false, false>(c[jj][4 * e], c[jj][4 * e + 1], c[jj][4 * e + 2], c[jj][4 * e + 3], c[jj][4 * e + 4],
                                          c[jj][4 * e + 5], c[jj][4 * e + 6], c[jj][4 * e + 7], eh[e]);
            }
#pragma unroll
            for (int r = 1; r < 20; ++r) {
                if constexpr (NH == 1) {
                    wy[r] = pack_cols(c[0][r], c[2 / NH - 1][r]);
                } else {                    // the other pair from the partner lane
                    const s2 o = as_s2(partner(as_w(c[0][r])));
                    wy[r] = h ? pack_cols(o, c[0][r]) : pack_cols(c[0][r], o);
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) U.y[r][4 * sc + q] = wy[4 + r];
        }
        if constexpr (DOC) {
            // chroma plane p, columns 4d .. 4d+3 (dword d), rows -2..7; the halves of a pair sit
            // in segments 2d and 2d+1 of luma H edge 0 / 2
#pragma unroll
            for (int r = 0; r < 2; ++r) wcv[r] = (uint32_t)rin[4 + r];
#pragma unroll
            for (int r = 0; r < 8; ++r) wcv[2 + r] = U.c[p][r][2 * sc + d];
            EdgeP eh[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) eh[e] = edge_params(cpar[e == 0 ? 1 : 2], bs_pair(inf[4 + 2 * e], 2 * d, 2 * d + 1));
            s2 c[2 / NH][10];
#pragma unroll
            for (int jj = 0; jj < 2 / NH; ++jj) {
                const int j = NH == 2 ? h : jj;
#pragma unroll
                for (int r = 0; r < 10; ++r) c[jj][r] = unpack_cols(wcv[r], j);
                s2 d0 = c[jj][0], d1 = c[jj][9];
                filter2<true, true>(d0, d0, c[jj][0], c[jj][1], c[jj][2], c[jj][3], d1, d1, eh[0]);
                filter2<false, true>(d0, d0, c[jj][4], c[jj][5], c[jj][6], c[jj][7], d1, d1, eh[1]);
            }
#pragma unroll
            for (int r = 1; r < 10; ++r) {
                if constexpr (NH == 1) {
                    wcv[r] = pack_cols(c[0][r], c[2 / NH - 1][r]);
                } else {
                    const s2 o = as_s2(partner(as_w(c[0][r])));
                    wcv[r] = h ? pack_cols(o, c[0][r]) : pack_cols(c[0][r], o);
                }
            }
#pragma unroll
            for (int r = 0; r < 8; ++r) U.c[p][r][2 * sc + d] = wcv[2 + r];
        }
        }

        // 7. publish / store what is final now: the 16 granules of MB x that MB x+1 cannot
        // change, four per lane; rows 13..15 (chroma 7) of MB (x, y-1)
#pragma unroll
        for (int jj = 0; jj < 2 / NH; ++jj) {
            const int j = NH == 2 ? h : jj;
            if constexpr (PL == 2)
                publish_pair(xok ? rec_out : OOB, max(x, 0), sc, early_c(q, j), early_k(q, j));
            else if constexpr (PL == 0)  // luma dwords 0..2: lanes (q < 3, h) publish pair h
                publish_pair(xok && q < 3 ? rec_out : OOB, max(x, 0), sc, q, h);
            else                         // chroma dword 0 (consumers 0, 2): lanes (q even, 0)
                publish_pair(xok && h == 0 && !(q & 1) ? rec_out : OOB, max(x, 0), sc, q, 2);
        }
        // rows 13..15 (chroma 7) of MB (x, y-1), final now: into the staging of the unit above, or
        // (the band's first row) into this unit's own
        if (xok && above) {
            if constexpr (DOY) {
                uint32_t* yd = rb ? &TA.y[13][x % SG][q] : &TU.yu[0][x % SG][q];
#pragma unroll
                for (int r = 1; r < 4; ++r) yd[(r - 1) * 4 * SG] = wy[r];
            }
            if constexpr (DOC) *(rb ? &TA.c[p][7][x % SG][d] : &TU.cu[p][x % SG][d]) = wcv[1];
        }
        // 8. what the next step fills: MB x+2 and its DbInfo
        fetch(x + 2);
        load_info(x + 2);
        wave_sync();                             // H(x) of every unit is in LDS
        TRACE({ const unsigned long long t2 = __builtin_amdgcn_s_memtime(); tph[3] += t2 - tm; tm = t2; })
    }
#if !(H264R_DB2_DIAG & 1)
    if (ok) {                            // the groups the last step completed
        wave_sync();
        store_groups(x - 1);
    }
#endif
    if (!ok) {
        // release the band below (the error is flagged)
        for (int m = 0; m < W; ++m)
            for (int k = 0; k < 3; ++k) {
                const v4u v = {0u, tag32, 0u, tag32};
                if (local) st16(hrs, pair_off(rec_out, m, q, k), v);
                else st16<AUX_SC1>(hrs, pair_off(rec_out, m, q, k), v);
            }
    }
    // (indexed band-major over (band, group) whatever the XCD-local ticket numbering)
    TRACE(const int tix = band * ngroups + grp;
          if (lane == 0 && tix < (1 << 16)) {
        h264r_db2_trace[tix][0] = tr_start; h264r_db2_trace[tix][1] = __builtin_amdgcn_s_memrealtime();
        for (int i = 0; i < 4; ++i) h264r_db2_trace[tix][2 + i] = tph[i];
        h264r_db2_trace[tix][6] = (unsigned long long)W; })
    }
}
