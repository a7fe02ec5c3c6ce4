// h264r_host.hip -- the C ABI of include/h264r.h on top of the gfx950 kernels.
//
// Host-side replacement of vio::h264::Decoder (decoder.h:301-338):
//   picture_begin / mb_submit / picture_end   ~ Decoder::init, decode(mb), deblock_filter
//   decode_batch                              ~ decode + deblock_filter of many pictures at once
// The reconstruction itself never runs on the CPU: every entry point that
// produces samples launches k_inter / k_intra / k_deblock and fails with
// H264R_ENODEVICE when no gfx950 device is present.
//
// Launch sequence per batch: k_inter (every inter / PCM MB, fully parallel),
// k_intra_pic (intra MBs, banded workgroups walking the wavefront),
// k_deblock (deblocking, one wave per pair of MB rows walking the wavefront).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "h264r.h"
#include "launch_cfg.h"

#ifndef H264R_WALK_ROWS
#define H264R_WALK_ROWS 8       // k_intra_pic: MB rows per band = waves per workgroup (k_picture.hip)
#endif

namespace h264r { struct DbInfo; }
extern "C" __global__ void k_inter4r(h264r_batch b, h264r::DbInfo* dbinfo, int2 rows, int* sp_flag, uint8_t* recon, int tag,
                                     int* zero, int nz, int* zero2, int nz2);
extern "C" __global__ void k_inter_sp(h264r_batch b, int2 rows, const int* sp_flag, uint8_t* recon, int tag);
extern "C" __global__ void k_derive444(h264r_batch b, int pl, int qpl, h264r_mb* mbs, h264r_slice* slices, h264r_quant* quant,
                                       const uint8_t** refs, int ntab, int* err);
extern "C" __global__ void k_untile(h264r_batch b, int2 rows, const uint8_t* recon);
extern "C" __global__ void k_c422_inter(h264r_batch b, int2 rows, int* err);
extern "C" __global__ void k_c422_intra(h264r_batch b, int2 rows, int* err);
extern "C" __global__ void k_c422_db(h264r_batch b, const h264r::DbInfo* dbinfo, int2 rows, int* err);
extern "C" __global__ void k_mbaff_inter(h264r_batch b, int* err);
extern "C" __global__ void k_mbaff_intra(h264r_batch b, int diag, int* err);
extern "C" __global__ void k_mbaff_deblock(h264r_batch b, int diag, int* err);
extern "C" __global__ void k_intra_pic(h264r_batch b, int* sync, int* err, const uint16_t* lvl, int lmax, int2 rows,
                                      int gstep, uint8_t* recon, const int* pband);
extern "C" __global__ void k_level(h264r_batch b, uint16_t* lvl, int* lvsync, int* lcount, int2 rows, int deep_cut,
                                   int lmax, int* pband);
extern "C" __global__ void k_level_scatter(h264r_batch b, const uint16_t* lvl, const int* lcount, int* lbase, int* lcursor,
                                           uint32_t* list, int2 rows);
extern "C" __global__ void k_intra_levels(h264r_batch b, const int* lcount, const int* lbase, const uint32_t* list,
                                          int lmax, int* lvsync, int* err, uint8_t* recon, int* bar);
constexpr int LEVEL_MAX_MBS = 65536;      // k_level's LDS bitmap (k_picture.hip)
constexpr int LEVEL_LDS = 40960;          // k_level's LDS level bytes: (W + 2) x (rows + 1) (k_picture.hip)
constexpr int LEVEL_LISTS = 64;           // levels with MB lists (H264R_LEVEL_LISTS, k_picture.hip)
constexpr int LEVEL_IDS = 2 * (LEVEL_LISTS + 1);   // two lists per level (k_picture.hip LEVEL_IDS)
extern "C" __global__ void k_deblock(h264r_batch b, const h264r::DbInfo* dbinfo, uint64_t* hb,
                                     int* sync, int* err, uint32_t epoch, int2 rows, int nx, uint8_t* recon);
extern "C" __global__ void k_deblock2(h264r_batch b, const h264r::DbInfo* dbinfo, uint64_t* hb,
                                      int* sync, int* err, uint32_t epoch, int2 rows, int nx, const uint8_t* recon);
extern "C" __global__ void k_deblock2y(h264r_batch b, const h264r::DbInfo* dbinfo, uint64_t* hb,
                                      int* sync, int* err, uint32_t epoch, int2 rows, int nx, const uint8_t* recon);
extern "C" __global__ void k_deblock2c(h264r_batch b, const h264r::DbInfo* dbinfo, uint64_t* hb,
                                      int* sync, int* err, uint32_t epoch, int2 rows, int nx, const uint8_t* recon);
constexpr size_t DBINFO_BYTES = 80;
constexpr size_t HANDOFF_BYTES = 256;   // one tagged record (32 x {dword, epoch}) per MB
constexpr size_t HANDOFF2_BYTES = 384;  // k_deblock2: 2 row slots x 24 x {dword, tag} per MB column
constexpr int DEBLOCK2_UNITS = 64 / H264R_DB2_LPU;   // k_deblock2: (picture, MB row) units per wave (mb_deblock.h)
constexpr int DEBLOCK2_PICS = DEBLOCK2_UNITS / H264R_DB2_BAND;   // pictures per wave

namespace {

#define HIP_OK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
        fprintf(stderr, "h264r: %s failed: %s\n", #x, hipGetErrorString(e_)); return H264R_EDEVICE; } } while (0)

const int dequant_coef[6][3] = {{10, 13, 16}, {11, 14, 18}, {13, 16, 20}, {14, 18, 23}, {16, 20, 25}, {18, 23, 29}};
const int dq8_v[6][6] = {{20, 18, 32, 19, 25, 24}, {22, 19, 35, 21, 28, 26}, {26, 23, 42, 24, 33, 31},
                         {28, 25, 45, 26, 35, 33}, {32, 28, 51, 30, 40, 38}, {36, 32, 58, 34, 46, 43}};

// normative LevelScale(m, i, j) (transform.cc:93-170 tables dequant_coef / dequant_coef8)
int norm4(int m, int i, int j)
{
    if ((i & 1) == 0 && (j & 1) == 0) return dequant_coef[m][0];
    if ((i & 1) && (j & 1)) return dequant_coef[m][2];
    return dequant_coef[m][1];
}
int norm8(int m, int i, int j)
{
    if (i % 4 == 0 && j % 4 == 0) return dq8_v[m][0];
    if (i % 2 == 1 && j % 2 == 1) return dq8_v[m][1];
    if (i % 4 == 2 && j % 4 == 2) return dq8_v[m][2];
    if ((i % 4 == 0 && j % 2 == 1) || (i % 2 == 1 && j % 4 == 0)) return dq8_v[m][3];
    if ((i % 4 == 0 && j % 4 == 2) || (i % 4 == 2 && j % 4 == 0)) return dq8_v[m][4];
    return dq8_v[m][5];
}

int grid_diag(int step, int W, int H)
{
    int ymin = step - (W - 1) > 0 ? (step - (W - 1) + 1) / 2 : 0;
    int ymax = std::min(step / 2, H - 1);
    return ymax >= ymin ? ymax - ymin + 1 : 0;
}

template <typename T>
int dev_resize(T** p, size_t* cap, size_t n)
{
    if (n <= *cap && *p) return H264R_OK;
    // work still queued may read the old buffer (h264r_picture_end_async): drain it first
    if (*p) { (void)hipDeviceSynchronize(); (void)hipFree(*p); }
    *p = nullptr; *cap = 0;
    if (hipMalloc(reinterpret_cast<void**>(p), std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return H264R_ENOMEM;
    *cap = n;
    return H264R_OK;
}

}  // namespace

// Per-batch scratch of one launch sequence.
struct Scratch {
    uint8_t* d_dbinfo = nullptr; size_t c_dbinfo = 0;
    int* d_sync = nullptr; size_t c_sync = 0;
    int tag = 0;                    // launch-sequence tag (> 0): k_inter4r's SP word
    uint8_t* d_hb = nullptr; size_t c_hb = 0;
    uint32_t epoch = 0;             // tag of the deblocking hand-off records of the last launch
    uint8_t* d_hb2 = nullptr; size_t c_hb2 = 0;
    uint32_t epoch2 = 0;            // the same for k_deblock2 (< 2^20: its tags carry the row)
    uint16_t* d_lvl = nullptr; size_t c_lvl = 0;   // intra dependency level per MB
    uint32_t* d_list = nullptr; size_t c_list = 0; // intra MBs by level (pic * nmb + addr)
    int* d_lcnt = nullptr; size_t c_lcnt = 0;      // [count | base | cursor] x LEVEL_IDS
    uint8_t* d_recon = nullptr; size_t c_recon = 0; // MB-tiled reconstruction, 384 B per (picture, MB)
    void release()
    {
        void* bufs[] = {d_dbinfo, d_sync, d_hb, d_hb2, d_lvl, d_list, d_lcnt, d_recon};
        for (void* b : bufs) if (b) (void)hipFree(b);
    }
};

struct h264r_ctx {
    int device = 0;
    int max_w = 0, max_h = 0;
    int fmt = 1;                          // chroma_format_idc: 1 (4:2:0), 0 (4:0:0) / 2 (4:2:2) (run_422) or 3 (4:4:4, run_444)
    // 4:4:4: one colour plane's derived batch (k_derive444) -- records, slices, quant, DPB tables --
    // and the scratch its unused 4:2:0 chroma outputs go to
    h264r_mb* d444_mbs = nullptr; size_t c444_mbs = 0;
    h264r_slice* d444_slices = nullptr; size_t c444_slices = 0;
    h264r_quant* d444_quant = nullptr; size_t c444_quant = 0;
    const uint8_t** d444_refs = nullptr; size_t c444_refs = 0;
    uint8_t* d444_chroma = nullptr; size_t c444_chroma = 0;
    hipStream_t stream = nullptr;
    // DPB slots
    uint8_t* slot[H264R_MAX_SLOTS][3] = {};
    int slot_w[H264R_MAX_SLOTS] = {}, slot_h[H264R_MAX_SLOTS] = {};
    const uint8_t** d_ref_planes = nullptr;
    int* d_err = nullptr;                 // [0] device error word (a bounded wait expired), [1] wait bound
    uint32_t wait_ticks = 0;              // err[1] as last written (s_memrealtime ticks, 100 MHz)
    uint32_t wait_val = 0;                // its host copy, the source of the async write
    // streaming-API staging: two pictures, so that one is parsed (h264r_picture_begin /
    // h264r_mb_submit) while the other is reconstructed (h264r_picture_end_async)
    struct StreamPic {
        int pw = 0, ph = 0;
        std::vector<h264r_mb> h_mbs;
        std::vector<int16_t> h_levels;
        std::vector<uint32_t> h_mv;
        std::vector<int8_t> h_ref;
        std::vector<h264r_slice> h_slices;
        h264r_pic h_pic{};
        h264r_quant h_quant{};
        std::vector<uint8_t> seen;
        uint8_t* out = nullptr; size_t c_out = 0;   // pinned planes Y | Cb | Cr, then the error word
        hipEvent_t done = nullptr;                 // its uploads, launches and readback
        bool pending = false;
    };
    StreamPic sp[2];
    int sp_fill = 0, sp_wait = 0, sp_pending = 0;
    bool in_pic = false;
    // device buffers of the streaming API
    h264r_mb* d_mbs = nullptr; size_t c_mbs = 0;
    int16_t* d_levels = nullptr; size_t c_levels = 0;
    uint32_t* d_mv = nullptr; size_t c_mv = 0;
    int8_t* d_ref = nullptr; size_t c_ref = 0;
    h264r_slice* d_slices = nullptr; size_t c_slices = 0;
    h264r_pic* d_pic = nullptr; size_t c_pic = 0;
    h264r_quant* d_quant = nullptr; size_t c_quant = 0;
    uint8_t* d_out = nullptr; size_t c_out = 0;
    // per-batch scratch of the launch sequence
    Scratch sc;
    int levels_grid = 0;                           // resident workgroups of k_intra_levels
    int nxcc = 0;                                  // XCDs of the device (k_deblock2's placement)
    // the per-batch scratch above is reused by every launch: a launch on a stream other
    // than the previous one first waits for the previous launch (ev_last)
    hipStream_t last_stream = nullptr;
    hipEvent_t ev_last = nullptr;
    // the overlapped schedule (launch_all): deblocking of picture chunk k on `side` while the
    // launch stream reconstructs chunk k + 1; ev_chunk[k] = chunk k reconstructed, ev_side =
    // the side stream's last deblocking launch (the launch stream waits for it at the end)
    hipStream_t side = nullptr;
    std::vector<hipEvent_t> ev_chunk;
    hipEvent_t ev_side = nullptr;
    hipEvent_t ev_fork = nullptr;              // the split deblocking walk: launch stream -> side stream
    // timing: every kernel of every launch bracketed by events on its stream
    bool timing = false;
    int debug = 0;
    struct Span { int kind; hipEvent_t a, b; };
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    std::vector<Span> spans;
    int timed_launches = 0;
};

extern "C" {

int h264r_abi_version(void) { return H264R_ABI_VERSION; }

const char* h264r_strerror(int s)
{
    switch (s) {
    case H264R_OK: return "ok";
    case H264R_EINVAL: return "invalid argument";
    case H264R_ENOMEM: return "out of memory";
    case H264R_EDEVICE: return "HIP runtime error";
    case H264R_ESTATE: return "call out of order";
    case H264R_EUNSUPPORTED: return "unsupported configuration";
    case H264R_ENODEVICE: return "no gfx950 device";
    default: return "unknown status";
    }
}

int h264r_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    int ok = 0;
    for (int d = 0; d < n; ++d) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, d) == hipSuccess && strncmp(p.gcnArchName, "gfx950", 6) == 0) ++ok;
    }
    return ok;
}

int h264r_quant_init_flat(h264r_quant* q)
{
    if (!q) return H264R_EINVAL;
    for (int t = 0; t < 2; ++t)
        for (int pl = 0; pl < 3; ++pl)
            for (int m = 0; m < 6; ++m) {
                for (int k = 0; k < 16; ++k) q->scale4x4[t][pl][m][k] = (int16_t)(norm4(m, k / 4, k % 4) * 16);
                for (int k = 0; k < 64; ++k) q->scale8x8[t][pl][m][k] = (int16_t)(norm8(m, k / 8, k % 8) * 16);
            }
    return H264R_OK;
}

int h264r_quant_init_lists(h264r_quant* q, const int32_t* const qm[12])
{
    // Transform::set_quant (transform.cc:259-302): InvLevelScale = dequant_coef x qmatrix.
    if (!q || !qm) return H264R_EINVAL;
    for (int i = 0; i < 12; ++i) if (!qm[i]) return H264R_EINVAL;
    for (int pl = 0; pl < 3; ++pl)
        for (int m = 0; m < 6; ++m) {
            for (int k = 0; k < 16; ++k) {
                q->scale4x4[0][pl][m][k] = (int16_t)(norm4(m, k / 4, k % 4) * qm[pl][k]);
                q->scale4x4[1][pl][m][k] = (int16_t)(norm4(m, k / 4, k % 4) * qm[3 + pl][k]);
            }
            for (int k = 0; k < 64; ++k) {
                // 8x8 lists: 6 Intra Y, 7 Inter Y, 8 Intra Cb, 9 Inter Cb, 10 Intra Cr, 11 Inter Cr
                q->scale8x8[0][pl][m][k] = (int16_t)(norm8(m, k / 8, k % 8) * qm[6 + 2 * pl][k]);
                q->scale8x8[1][pl][m][k] = (int16_t)(norm8(m, k / 8, k % 8) * qm[7 + 2 * pl][k]);
            }
        }
    return H264R_OK;
}

// Environment knobs, read and validated once (at the first h264r_create).  Each one only
// chooses between bit-exact schedules or bounds a wait; a value out of its range fails
// h264r_create with H264R_EINVAL (stderr names it) instead of being taken for another setting.
struct Knobs {
    bool ok = true;
    int debug = 0;             // H264R_DEBUG: schedule flags of h264r_set_debug OR-ed into every launch
    uint32_t wait_ticks = 0;   // H264R_WAIT_MS: bound of every device-side wait (below)
    int levels = -1;           // H264R_LEVELS: dependency levels from lists (-1: by launch size, level_launches)
    int deblock2_min = 8;      // H264R_DEBLOCK2_MIN: batches of this many 68-row pictures' worth of MB rows deblock with k_deblock2
    int deblock2s_max = 512;   // H264R_DB2S_MAX: batches of fewer 68-row pictures' worth of MB rows take the split walk
    int lvl_margin = 1;        // H264R_LVL_MARGIN: k_intra_levels' grid, blocks per CU below occupancy
    bool coop = false;         // H264R_COOP: k_intra_levels by hipLaunchCooperativeKernel (1) or a plain launch
    int walk_gstep = 0;        // H264R_WALK_GSTEP: the walk's band hand-off period (0: by batch size)
    int overlap = 1;           // H264R_OVERLAP: picture chunks of the overlapped schedule (launch_all; 0, 1: off)
    bool verbose = false;      // H264R_VERBOSE
};
static bool env_long(const char* name, long lo, long hi, long* out)
{
    const char* e = getenv(name);
    if (!e) return true;
    char* end = nullptr;
    errno = 0;
    const long v = strtol(e, &end, 10);
    if (end == e || *end != '\0' || errno != 0 || v < lo || v > hi) {
        fprintf(stderr, "h264r: %s=\"%s\" is not an integer in [%ld, %ld]\n", name, e, lo, hi);
        return false;
    }
    *out = v;
    return true;
}
constexpr int SCHEDULE_FLAGS = H264R_DBG_INTRA_WALK | H264R_DBG_DEBLOCK_MB | H264R_DBG_DEBLOCK_ROWS | H264R_DBG_DEBLOCK_GLOBAL |
                               H264R_DBG_OVERLAP | H264R_DBG_DEBLOCK_SPLIT;
static const Knobs& knobs()
{
    static const Knobs k = [] {
        Knobs n;
        long v;
        // flags that change or skip work (H264R_DBG_NO_DEBLOCK, the wait test) are API-only
        v = 0; n.ok &= env_long("H264R_DEBUG", 0, SCHEDULE_FLAGS, &v);
        if (v & ~SCHEDULE_FLAGS) { fprintf(stderr, "h264r: H264R_DEBUG=%ld: only schedule flags (%d)\n", v, SCHEDULE_FLAGS); n.ok = false; }
        n.debug = (int)(v & SCHEDULE_FLAGS);
        // a launch of the slowest kernel over the largest batch takes ~10 ms, and a wait only
        // ever waits on work that is already running: 2 s means a lost wave
        v = 2000; n.ok &= env_long("H264R_WAIT_MS", 1, 40000, &v);
        n.wait_ticks = (uint32_t)(v * 100000);                     // s_memrealtime, 100 MHz
        // levels beyond 3 hold few MBs each, and a grid barrier apiece: the walk takes them
        v = -1; n.ok &= env_long("H264R_LEVELS", 0, LEVEL_LISTS, &v); n.levels = (int)v;
        // round 5 (8 lanes per unit, staged stores): k_deblock2 wins over k_deblock from 64 1080p
        // pictures of a throughput batch, 32 2160p chain pictures, up (profiles/r05_x_deblock_min.txt).
        // Below H264R_DB2S_MAX the split walk is the default, so k_deblock is taken by default only
        // when H264R_DB2S_MAX is lowered (0: launches below this many picture-rows x 68 take it)
        v = 8; n.ok &= env_long("H264R_DEBLOCK2_MIN", 1, 1L << 30, &v); n.deblock2_min = (int)v;
        // the split walk (twice the waves, each step shorter) wins below ~512 1080p pictures: config 3
        // at 128 / 256 / 1024 pictures 1.06 -> 0.83 / 1.26 -> 1.23 / 3.78 -> 4.46 ms, config 4 (256)
        // 1.28 -> 1.22, config 5 (64 2160p) 2.07 -> 1.66, the latency chain and chain mode
        // (profiles/r05_ak_split_walk_ab.txt)
        v = 512; n.ok &= env_long("H264R_DB2S_MAX", 0, 1L << 30, &v); n.deblock2s_max = (int)v;
        v = 1; n.ok &= env_long("H264R_LVL_MARGIN", 0, 7, &v); n.lvl_margin = (int)v;
        // a plain launch by default: the same throughput and latency as the cooperative one
        // (profiles/r05_w_chain_coop.txt), and the launch rocprofv3 can profile (it crashes at exit
        // after a cooperative launch), so the profiled sequence is the benchmarked one
        v = 0; n.ok &= env_long("H264R_COOP", 0, 1, &v); n.coop = v != 0;
        v = 0; n.ok &= env_long("H264R_WALK_GSTEP", 0, 1 << 20, &v); n.walk_gstep = (int)v;
        // measured slower than one stage (profiles/r05_b_overlap_ab.txt): off by default
        v = 1; n.ok &= env_long("H264R_OVERLAP", 0, 16, &v); n.overlap = (int)v;
        v = 0; n.ok &= env_long("H264R_VERBOSE", 0, 1, &v); n.verbose = v != 0;
        return n;
    }();
    return k;
}
static uint32_t wait_bound_ticks() { return knobs().wait_ticks; }
// err[1] is rewritten in stream order on the launch stream s (a launch still running on
// another stream keeps the bound it started with only if it is ordered before -- run_batch
// orders every launch of the context after the previous one)
static int set_wait_bound(h264r_ctx* c, uint32_t ticks, hipStream_t s)
{
    if (c->wait_ticks == ticks) return H264R_OK;
    c->wait_val = ticks;
    HIP_OK(hipMemcpyAsync(c->d_err + 1, &c->wait_val, sizeof(uint32_t), hipMemcpyHostToDevice, s));
    c->wait_ticks = ticks;
    return H264R_OK;
}

int h264r_create(h264r_ctx** out, int device, int max_w, int max_h, int chroma_format_idc, int bit_depth)
{
    if (!out || max_w <= 0 || max_h <= 0 || max_w > 1024 || max_h > 1024) return H264R_EINVAL;
    *out = nullptr;
    if (!knobs().ok) return H264R_EINVAL;            // an environment knob out of range (stderr)
    if (chroma_format_idc < 0 || chroma_format_idc > 3 || bit_depth != 8) return H264R_EUNSUPPORTED;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) return H264R_ENODEVICE;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess || strncmp(p.gcnArchName, "gfx950", 6) != 0)
        return H264R_ENODEVICE;
    h264r_ctx* c = new (std::nothrow) h264r_ctx();
    if (!c) return H264R_ENOMEM;
    c->device = device; c->max_w = max_w; c->max_h = max_h; c->fmt = chroma_format_idc;
    // the context's own stream is a BLOCKING stream: work on the legacy NULL stream (torch's
    // default stream) and this stream are ordered with each other
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamDefault) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&c->d_ref_planes), sizeof(uint8_t*) * 3 * H264R_MAX_SLOTS) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&c->d_err), 2 * sizeof(int)) != hipSuccess) {
        delete c;
        return H264R_EDEVICE;
    }
    if (hipEventCreateWithFlags(&c->ev_last, hipEventDisableTiming) != hipSuccess) { delete c; return H264R_EDEVICE; }
    (void)hipMemset(c->d_ref_planes, 0, sizeof(uint8_t*) * 3 * H264R_MAX_SLOTS);
    (void)hipMemset(c->d_err, 0, 2 * sizeof(int));
    if (set_wait_bound(c, wait_bound_ticks(), c->stream) != H264R_OK || hipStreamSynchronize(c->stream) != hipSuccess) {
        (void)h264r_destroy(c);
        return H264R_EDEVICE;
    }
    *out = c;
    return H264R_OK;
}

int h264r_destroy(h264r_ctx* c)
{
    if (!c) return H264R_EINVAL;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (int s = 0; s < H264R_MAX_SLOTS; ++s) if (c->slot[s][0]) (void)hipFree(c->slot[s][0]);
    void* bufs[] = {c->d_ref_planes, c->d_err, c->d_mbs, c->d_levels, c->d_mv, c->d_ref, c->d_slices, c->d_pic, c->d_quant, c->d_out,
                    c->d444_mbs, c->d444_slices, c->d444_quant, c->d444_refs, c->d444_chroma};
    for (void* b : bufs) if (b) (void)hipFree(b);
    for (auto& p : c->sp) {
        if (p.out) (void)hipHostFree(p.out);
        if (p.done) (void)hipEventDestroy(p.done);
    }
    c->sc.release();
    for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->ev_last) (void)hipEventDestroy(c->ev_last);
    if (c->side) (void)hipStreamSynchronize(c->side);
    for (hipEvent_t e : c->ev_chunk) (void)hipEventDestroy(e);
    if (c->ev_side) (void)hipEventDestroy(c->ev_side);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return H264R_OK;
}

// Bytes of one chroma plane of a w x h MB picture: 8 x 8 samples per MB (4:2:0), 8 x 16 (4:2:2)
// or 16 x 16 (4:4:4).
static size_t chroma_bytes(const h264r_ctx* c, int w, int h)
{
    return (size_t)w * h * (c->fmt == 3 ? 256 : c->fmt == 2 ? 128 : c->fmt == 1 ? 64 : 0);     // 4:0:0: none
}

static int ensure_slot(h264r_ctx* c, int slot, int w, int h)
{
    if (c->slot[slot][0] && c->slot_w[slot] == w && c->slot_h[slot] == h) return H264R_OK;
    if (c->slot[slot][0]) {
        (void)hipDeviceSynchronize();
        (void)hipFree(c->slot[slot][0]);
        c->slot[slot][0] = nullptr;
    }
    size_t ys = (size_t)w * 16 * h * 16, cs = chroma_bytes(c, w, h);
    uint8_t* base = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&base), ys + 2 * cs + H264R_PLANE_SLACK) != hipSuccess) return H264R_ENOMEM;
    c->slot[slot][0] = base; c->slot[slot][1] = base + ys; c->slot[slot][2] = base + ys + cs;
    c->slot_w[slot] = w; c->slot_h[slot] = h;
    HIP_OK(hipMemcpy(c->d_ref_planes + 3 * slot, c->slot[slot], 3 * sizeof(uint8_t*), hipMemcpyHostToDevice));
    return H264R_OK;
}

int h264r_set_ref(h264r_ctx* c, int slot, const uint8_t* y, const uint8_t* u, const uint8_t* v, int w, int h)
{
    if (!c || slot < 0 || slot >= H264R_MAX_SLOTS || !y || (c->fmt && (!u || !v)) || w <= 0 || h <= 0 ||
        w > c->max_w || h > c->max_h)
        return H264R_EINVAL;
    (void)hipSetDevice(c->device);
    int st = ensure_slot(c, slot, w, h);
    if (st) return st;
    size_t ys = (size_t)w * 16 * h * 16, cs = chroma_bytes(c, w, h);
    HIP_OK(hipMemcpyAsync(c->slot[slot][0], y, ys, hipMemcpyHostToDevice, c->stream));
    if (cs) {
        HIP_OK(hipMemcpyAsync(c->slot[slot][1], u, cs, hipMemcpyHostToDevice, c->stream));
        HIP_OK(hipMemcpyAsync(c->slot[slot][2], v, cs, hipMemcpyHostToDevice, c->stream));
    }
    HIP_OK(hipStreamSynchronize(c->stream));
    return H264R_OK;
}

int h264r_ref_planes(h264r_ctx* c, int slot, uint8_t** y, uint8_t** u, uint8_t** v)
{
    if (!c || slot < 0 || slot >= H264R_MAX_SLOTS) return H264R_EINVAL;
    if (y) *y = c->slot[slot][0];
    if (u) *u = c->slot[slot][1];
    if (v) *v = c->slot[slot][2];
    return c->slot[slot][0] ? H264R_OK : H264R_ESTATE;
}

static hipEvent_t timing_event(h264r_ctx* c)
{
    if (c->ev_used == c->ev_pool.size()) {
        hipEvent_t e = nullptr;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        c->ev_pool.push_back(e);
    }
    return c->ev_pool[c->ev_used++];
}

// Bracket one launch with timing events on its stream (kind: 0 prep+inter, 1 intra,
// 2 deblock, 3 whole batch).
struct Timed {
    h264r_ctx* c; int kind; hipStream_t s; hipEvent_t a = nullptr;
    Timed(h264r_ctx* c_, int k, hipStream_t s_) : c(c_), kind(k), s(s_)
    {
        if (c && c->timing && (a = timing_event(c))) (void)hipEventRecord(a, s);
    }
    ~Timed()
    {
        if (!a) return;
        hipEvent_t b = timing_event(c);
        if (b) { (void)hipEventRecord(b, s); c->spans.push_back({kind, a, b}); }
    }
};

// Intra MBs are scheduled by dependency level: k_level computes every MB's level and
// counts them, k_level_scatter builds one MB list per level, and
// k_intra_levels does levels 1..N from those lists in one persistent cooperative launch
// (a grid barrier between levels); the wavefront walk k_intra_pic takes whatever lies
// deeper.  N by default: 4 for launches of >= LEVELS4_MIN_MBS MBs, else 3.  P / B pictures
// rarely go deeper, and in all-intra pictures (levels x + 2y + 1) a level holds a few MBs per
// picture, so the walk's row-to-row hand-off beats one grid barrier per level (config 2: 36.6 ms
// of intra walking vs 44.9 with every level from lists).  A fourth level paid once the level
// barrier was sharded, on large launches only (round 5, profiles/r05_aw_levels4_ab.txt: config
// 3's 1024 pictures intra 1.215 -> 1.148 ms; config 4's 256 pictures 0.383 -> 0.411, chain
// mode config 4 0.148 -> 0.200).  H264R_LEVELS=<N> sets N (0: walk only; at most LEVEL_LISTS).
constexpr size_t LEVELS4_MIN_MBS = (size_t)4 << 20;
static int level_launches(size_t mbs)
{
    const int v = knobs().levels;
    return v >= 0 ? v : mbs >= LEVELS4_MIN_MBS ? 4 : 3;
}

// Pictures [p0, p0 + n) of a batch as a batch of their own: every per-picture array advanced
// (the level pool is shared: coef_off stays an offset into it).
static h264r_batch sub_batch(const h264r_batch& b, int p0, int n)
{
    h264r_batch r = b;
    const size_t nmb = (size_t)b.width_mbs * b.height_mbs;
    r.num_pics = n;
    r.mbs += (size_t)p0 * nmb;
    r.mv += (size_t)p0 * 32 * nmb;                 // [list][4H][4W] per picture
    r.ref_idx += (size_t)p0 * 32 * nmb;
    r.slices += (size_t)p0 * b.slice_stride;
    r.pics += p0;
    r.quant += p0;
    if (b.ref_planes_stride) r.ref_planes += (size_t)p0 * b.ref_planes_stride;
    r.out_y += (size_t)p0 * 256 * nmb;
    r.out_u += (size_t)p0 * 64 * nmb;
    r.out_v += (size_t)p0 * 64 * nmb;
    return r;
}

// ints of one launch sequence's sync region: [intra ticket + per-(picture, row) progress]
// [deblock ticket][level barrier, deepest level][2 unused] + the deblocking kernels' per-XCD
// ticket counters and done count (two sets: the split walk's luma and chroma kernels run
// together) + k_intra_levels' sharded grid barrier (8 shard counters + top) -- these 1 + P H + 32
// are zeroed by k_inter4r -- then per picture the walk's bands holding an MB deeper than the
// level lists (k_level -> k_intra_pic), and last the SP tag word (k_inter4r stores the launch
// tag when it met an inter MB of an SP slice).
static size_t sync_ints(int P, int H) { return 1 + (size_t)P * H + 32 + (size_t)P + 1; }

// One launch sequence's share of the scratch (the whole batch, or one chunk of the overlapped
// schedule): its pictures, their deblocking records and MB-tiled reconstruction, its sync region.
struct Stage {
    h264r_batch b;
    h264r::DbInfo* dbinfo;
    uint8_t* recon;
    int* sync;
};

// The reconstruction of a stage on stream s: k_inter4r + k_inter_sp (the deblocking records and
// the inter / PCM MBs), k_level + k_level_scatter + k_intra_levels +
// k_intra_pic (intra MBs).  The level lists are one set: stages on one stream reuse them in order.
static int recon_launches(h264r_ctx* c, const Stage& S, hipStream_t s, int2 rows, Scratch& X, bool levels, bool coop)
{
    const Knobs& K = knobs();
    const h264r_batch& b = S.b;
    const int W = b.width_mbs, H = b.height_mbs, P = b.num_pics, HB = rows.y - rows.x;
    const int nbands = (HB + H264R_WALK_ROWS - 1) / H264R_WALK_ROWS;
    const bool wait_test = (c->debug & H264R_DBG_WAIT_TEST) != 0;
    int* sync = S.sync;
    uint8_t* recon = S.recon;
    const int groups = (W * HB + 15) / 16;
    // groups per workgroup (launch_cfg.h), 8 XCD bands (k_recon.hip inter4_groups)
    const dim3 igrid(8 * ((groups + 8 * H264R_INTER_GROUPS - 1) / (8 * H264R_INTER_GROUPS)), P);
    {
        Timed t(c, 0, s);
        int* sp_flag = sync + 1 + (size_t)P * H + 32 + P;    // not zeroed: compared with the tag
        // the deblocking records and the inter / I_PCM reconstruction in one launch, which also
        // zeroes the stage's sync words and the level counters
        if (++X.tag <= 0) X.tag = 1;
        hipLaunchKernelGGL(k_inter4r, igrid, dim3(256), 0, s, b, S.dbinfo, rows, sp_flag, recon, X.tag, sync,
                           (int)(1 + (size_t)P * H + 32), levels ? X.d_lcnt : nullptr, levels ? 3 * LEVEL_IDS : 0);
        HIP_OK(hipGetLastError());
        // inter MBs of SP slices (a short launch when the batch has none)
        hipLaunchKernelGGL(k_inter_sp, dim3(1024), dim3(256), 0, s, b, rows, (const int*)sp_flag, recon, X.tag);
        HIP_OK(hipGetLastError());
    }
    {
        Timed t(c, 1, s);
        uint16_t* lvl = levels ? X.d_lvl : nullptr;
        int* pband = sync + 1 + (size_t)P * H + 32;             // after the zeroed words
        int* lbar = sync + 1 + (size_t)P * H + 23;               // k_intra_levels' barrier (9 ints)
        const int lmax = levels ? level_launches((size_t)P * W * HB) : 0;
        if (knobs().verbose) fprintf(stderr, "h264r: %d intra levels from lists, %d pictures\n", lmax, P);
        if (levels) {
            int* lvsync = sync + 1 + (size_t)P * H + 2;
            int* lcount = X.d_lcnt;
            int* lbase = lcount + LEVEL_IDS;
            int* lcursor = lbase + LEVEL_IDS;
            // pictures deeper than 4 x lmax levels (all-intra) are left to the walk whole
            hipLaunchKernelGGL(k_level, dim3(P), dim3(1024), 0, s, b, lvl, lvsync, lcount, rows, 4 * lmax, lmax, pband);
            HIP_OK(hipGetLastError());
            hipLaunchKernelGGL(k_level_scatter, dim3(P), dim3(1024), 0, s, b, (const uint16_t*)lvl, (const int*)lcount, lbase,
                               lcursor, X.d_list, rows);
            HIP_OK(hipGetLastError());
            // the grid one block per CU below the occupancy answer, all resident at once (the grid
            // barrier's contract, include/h264r.h); a plain launch by default, H264R_COOP=1 a
            // cooperative one (the runtime then checks the residency, or refuses the launch)
            // small batches (the latency chain: one picture) take a grid sized to their MBs,
            // 64 per workgroup: most workgroups of the full grid would only attend the grid
            // barriers, whose cost grows with the number of arrivals (MI355X_MICROARCH.md
            // price list 'barrier-xcd')
            const int lgrid = std::min(c->levels_grid, std::max(8, (int)(((size_t)P * W * HB + 63) / 64)));
            if (coop) {
                const int* lcount_c = lcount;
                const int* lbase_c = lbase;
                const uint32_t* list_c = X.d_list;
                int lmax_v = lmax;
                int* err_p = c->d_err;
                h264r_batch bv = b;
                void* args[] = {(void*)&bv, (void*)&lcount_c, (void*)&lbase_c, (void*)&list_c, (void*)&lmax_v,
                                (void*)&lvsync, (void*)&err_p, (void*)&recon, (void*)&lbar};
                HIP_OK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_intra_levels), dim3(lgrid),
                                                  dim3(256), args, 0, s));
            } else {
                hipLaunchKernelGGL(k_intra_levels, dim3(lgrid), dim3(256), 0, s, b, (const int*)lcount,
                                   (const int*)lbase, (const uint32_t*)X.d_list, lmax, lvsync, c->d_err, recon, lbar);
                HIP_OK(hipGetLastError());
            }
        }
        // the walk's band-to-band hand-off: global progress every gstep MBs (k_picture.hip);
        // H264R_WALK_GSTEP overrides
        const int gstep = wait_test ? -1 : K.walk_gstep > 0 ? K.walk_gstep : (P >= 128 ? 64 : 1);
        hipLaunchKernelGGL(k_intra_pic, dim3(P * nbands), dim3(64 * H264R_WALK_ROWS), 0, s, b, sync, c->d_err,
                           (const uint16_t*)lvl, lmax, rows, gstep, recon, (const int*)pband);
        HIP_OK(hipGetLastError());
    }
    return H264R_OK;
}

// The deblocking of a stage on stream s (sched 1 k_deblock2, 2 the split walk: k_deblock2y on s
// beside k_deblock2c on the context's side stream, 0 k_deblock), or the
// untiled copy of its reconstruction (H264R_DBG_NO_DEBLOCK).
static int deblock_launch(h264r_ctx* c, const Stage& S, hipStream_t s, int2 rows, uint8_t* hb, uint32_t epoch, int sched)
{
    const h264r_batch& b = S.b;
    const int W = b.width_mbs, H = b.height_mbs, P = b.num_pics, HB = rows.y - rows.x;
    const int npairs = (HB + 1) / 2;
    int* dsync = S.sync + 1 + (size_t)P * H + 5;
    if (c->debug & H264R_DBG_NO_DEBLOCK) {
        hipLaunchKernelGGL(k_untile, dim3((W * HB * 32 + 255) / 256, P), dim3(256), 0, s, b, rows, (const uint8_t*)S.recon);
        HIP_OK(hipGetLastError());
        return H264R_OK;
    }
    Timed t(c, 2, s);
    if (!c->nxcc) {                  // XCDs of the device: the deblocking kernels' placement
        int nx = 1;
        if (hipDeviceGetAttribute(&nx, hipDeviceAttributeNumberOfXccs, c->device) != hipSuccess) nx = 1;
        c->nxcc = std::max(1, std::min(nx, 8));
    }
    if (sched == 1 && knobs().verbose) {
        static bool once = false;
        int per_cu = 0;
        if (!once && hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k_deblock2), 64, 0) == hipSuccess)
            fprintf(stderr, "h264r: k_deblock2 occupancy %d waves/CU\n", per_cu);
        once = true;
    }
    if (sched) {
        // k_deblock2 keeps a picture group on one XCD (g % nx): nx counters
        int grid = ((P + DEBLOCK2_PICS - 1) / DEBLOCK2_PICS) * ((HB + H264R_DB2_BAND - 1) / H264R_DB2_BAND);
        const int nx = grid >= 64 * c->nxcc && !(c->debug & H264R_DBG_DEBLOCK_GLOBAL) ? c->nxcc : 1;
        grid = (grid + nx - 1) / nx * nx;
        if (sched == 2) {
            // the split walk: the luma and chroma planes filter independently (deblock.cc:418-535
            // per plane), so each plane's walk is its own wave with the shorter step; the chroma
            // walk on the side stream, joined back before anything after the deblocking
            if (!c->side) HIP_OK(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
            if (!c->ev_fork) HIP_OK(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
            if (!c->ev_side) HIP_OK(hipEventCreateWithFlags(&c->ev_side, hipEventDisableTiming));
            HIP_OK(hipEventRecord(c->ev_fork, s));
            HIP_OK(hipStreamWaitEvent(c->side, c->ev_fork, 0));
            hipLaunchKernelGGL(k_deblock2c, dim3(grid), dim3(64), 0, c->side, b, S.dbinfo, reinterpret_cast<uint64_t*>(hb),
                               dsync + 9, c->d_err, epoch, rows, nx, (const uint8_t*)S.recon);
            HIP_OK(hipGetLastError());
            hipLaunchKernelGGL(k_deblock2y, dim3(grid), dim3(64), 0, s, b, S.dbinfo, reinterpret_cast<uint64_t*>(hb),
                               dsync, c->d_err, epoch, rows, nx, (const uint8_t*)S.recon);
            HIP_OK(hipGetLastError());
            HIP_OK(hipEventRecord(c->ev_side, c->side));
            HIP_OK(hipStreamWaitEvent(s, c->ev_side, 0));
            return H264R_OK;
        }
        hipLaunchKernelGGL(k_deblock2, dim3(grid), dim3(64), 0, s, b, S.dbinfo, reinterpret_cast<uint64_t*>(hb), dsync,
                           c->d_err, epoch, rows, nx, (const uint8_t*)S.recon);
    } else {
        // k_deblock keeps a picture's pairs on one XCD (p % nx): nx times the largest
        // XCD share of waves, so every XCD runs all its pairs at once
        const int nx = c->nxcc > 1 && !(c->debug & H264R_DBG_DEBLOCK_GLOBAL) ? c->nxcc : 1;
        const int grid = nx * ((P + nx - 1) / nx) * npairs;
        hipLaunchKernelGGL(k_deblock, dim3(grid), dim3(64), 0, s, b, S.dbinfo, reinterpret_cast<uint64_t*>(hb), dsync,
                           c->d_err, epoch, rows, nx, S.recon);
    }
    HIP_OK(hipGetLastError());
    return H264R_OK;
}

// rows [row0, row1): the MB rows of every picture this launch reconstructs and deblocks (the
// whole picture, or a slice-aligned band: h264r_decode_batch_rows).
//
// Two schedules, both bit-exact:
// * one stage: the reconstruction kernels, then the deblocking kernel, on stream s;
// * overlapped (H264R_OVERLAP=<chunks>, each of >= 64 whole 1080p pictures' worth of MB rows;
//   off by default: measured slower): the batch is cut into picture chunks; the launch stream reconstructs
//   chunk after chunk and the context's side stream deblocks chunk k (after an event) while
//   the launch stream reconstructs chunk k + 1, so the latency-bound deblocking walk shares
//   the CUs with the issue-bound reconstruction (the order the reference keeps per picture,
//   deblock.cc:537-552 after decoder.cc:65-79 of every MB, is kept: a picture is deblocked
//   after all its MBs are reconstructed).  The launch stream then waits for the side stream.
//   k_intra_levels takes a plain launch here: a cooperative launch waits for the device to be
//   otherwise idle, which would serialise the two streams.
static int launch_all(h264r_ctx* c, const h264r_batch& b, hipStream_t s, int row0, int row1, Scratch& X)
{
    const Knobs& K = knobs();
    // H264R_DEBUG: the deblocking-schedule flags of h264r_set_debug OR-ed into every launch
    // (measurement A/B; validated in knobs(): schedule flags only, so the output is unchanged)
    const int debug_saved = c->debug;
    c->debug |= K.debug;
    struct Restore { h264r_ctx* c; int d; ~Restore() { c->debug = d; } } restore{c, debug_saved};
    const int W = b.width_mbs, H = b.height_mbs, P = b.num_pics, HB = row1 - row0;
    const int2 rows = make_int2(row0, row1);
    const int npairs = (HB + 1) / 2;
    const size_t nmb = (size_t)W * H;
    const bool wait_test = (c->debug & H264R_DBG_WAIT_TEST) != 0;
    // chunks of the overlapped schedule: each of >= 64 x 68 picture-MB-rows
    int nch = (c->debug & H264R_DBG_OVERLAP) ? std::max(K.overlap, 4) : K.overlap;
    nch = std::min(nch, (int)std::min<int64_t>(P, (int64_t)P * HB / (64 * 68)));
    if (nch < 2 || wait_test || (c->debug & H264R_DBG_NO_DEBLOCK)) nch = 1;
    const int chunk_min = P / nch;
    int st;
    if ((st = dev_resize(&X.d_dbinfo, &X.c_dbinfo, (size_t)P * nmb * DBINFO_BYTES))) return st;
    // the reconstruction kernels write the MB-tiled samples (device_common.h), the
    // deblocking kernel (or k_untile) turns them into the output planes
    if ((st = dev_resize(&X.d_recon, &X.c_recon, (size_t)P * nmb * 384))) return st;
    // k_deblock2 needs many (picture group, band) walks in flight: H264R_DEBLOCK2_MIN is the
    // crossover measured on whole 1080p pictures (68 MB rows), so a launch qualifies by its
    // picture-rows (a 2160p picture counts twice, a 17-row slice band a quarter); the chunks of
    // the overlapped schedule all take the schedule of the smallest
    // the split walk (k_deblock2y + k_deblock2c: shorter steps, twice the waves) below
    // H264R_DB2S_MAX pictures' worth of rows (not under the overlapped schedule, which has the
    // side stream already)
    const int64_t prows = (int64_t)chunk_min * HB;
    const int sched = (c->debug & H264R_DBG_DEBLOCK_SPLIT)   ? (nch > 1 ? 1 : 2)
                    : (c->debug & H264R_DBG_DEBLOCK_ROWS)    ? 1
                    : (c->debug & H264R_DBG_DEBLOCK_MB)      ? 0
                    : prows < (int64_t)K.deblock2s_max * 68 && nch == 1 ? 2
                    : prows >= (int64_t)K.deblock2_min * 68  ? 1 : 0;
    const bool by_rows = sched != 0;                 // k_deblock2's hand-off records (both widths)
    // hand-off records of the chosen deblocking kernel, a region per picture; fresh memory or a
    // wrapping epoch restarts from zeroed records, so no record may carry a live tag
    uint8_t** hb = by_rows ? &X.d_hb2 : &X.d_hb;
    size_t* hcap = by_rows ? &X.c_hb2 : &X.c_hb;
    uint32_t* ep = by_rows ? &X.epoch2 : &X.epoch;
    const uint32_t ep_max = by_rows ? (1u << 20) - 2 - 16 : 0xFFFFFF00u;
    const size_t hb_pic = by_rows ? (size_t)W * HANDOFF2_BYTES : (size_t)npairs * W * HANDOFF_BYTES;
    {
        const size_t cap_before = *hcap;
        if ((st = dev_resize(hb, hcap, (size_t)P * hb_pic))) return st;
        if (*hcap != cap_before || *ep > ep_max) {
            HIP_OK(hipMemsetAsync(*hb, 0, *hcap, s));
            *ep = 0;
        }
    }
    const size_t sync_n = (size_t)nch * sync_ints(chunk_min + 1, H);
    {
        // each stage's k_inter4r zeroes its sync words; fresh memory is zeroed once, so no stale
        // inter flag can carry a live tag
        const size_t cap_before = X.c_sync;
        if ((st = dev_resize(&X.d_sync, &X.c_sync, sync_n))) return st;
        if (X.c_sync != cap_before) HIP_OK(hipMemsetAsync(X.d_sync, 0, X.c_sync * sizeof(int), s));
    }
    // H264R_DBG_WAIT_TEST: every intra-walk wait asks for progress no row reaches, under a
    // 10 ms bound -- the launch must drain and h264r_check report H264R_EDEVICE
    if ((st = set_wait_bound(c, wait_test ? 1000000u : wait_bound_ticks(), s))) return st;
    const bool levels = nmb <= LEVEL_MAX_MBS && (size_t)(W + 2) * (HB + 1) <= (size_t)LEVEL_LDS && level_launches(0) > 0 &&
                        !(c->debug & (H264R_DBG_INTRA_WALK | H264R_DBG_WAIT_TEST));
    if (levels && !c->levels_grid) {
        // every workgroup of the persistent level kernel must be resident at once: one
        // block per CU below what the occupancy query reports (MI355X_MICROARCH.md,
        // residency caveat), at least one per CU
        int per_cu = 0, cus = 0;
        HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k_intra_levels), 256, 0));
        HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
        c->levels_grid = std::max(1, per_cu - K.lvl_margin) * std::max(1, cus);
        if (K.verbose)
            fprintf(stderr, "h264r: k_intra_levels occupancy %d blocks/CU, %d CUs, grid %d\n", per_cu, cus, c->levels_grid);
    }
    if (levels && ((st = dev_resize(&X.d_lvl, &X.c_lvl, (size_t)P * nmb)) ||
                   (st = dev_resize(&X.d_list, &X.c_list, (size_t)P * nmb)) ||
                   (st = dev_resize(&X.d_lcnt, &X.c_lcnt, 3 * (size_t)LEVEL_IDS))))
        return st;
    if (nch > 1) {
        if (!c->side) HIP_OK(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
        if (!c->ev_side) HIP_OK(hipEventCreateWithFlags(&c->ev_side, hipEventDisableTiming));
        while ((int)c->ev_chunk.size() < nch) {
            hipEvent_t e = nullptr;
            HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            c->ev_chunk.push_back(e);
        }
    }
    Timed whole(c, 3, s);
    if (c->timing) c->timed_launches++;
    for (int k = 0, p0 = 0; k < nch; ++k) {
        const int n = P / nch + (k < P % nch ? 1 : 0);
        Stage S{nch > 1 ? sub_batch(b, p0, n) : b, reinterpret_cast<h264r::DbInfo*>(X.d_dbinfo + (size_t)p0 * nmb * DBINFO_BYTES),
                X.d_recon + (size_t)p0 * nmb * 384,
                X.d_sync + (size_t)k * sync_ints(chunk_min + 1, H)};
        if ((st = recon_launches(c, S, s, rows, X, levels, K.coop && nch == 1))) return st;
        hipStream_t ds = s;
        if (nch > 1) {
            HIP_OK(hipEventRecord(c->ev_chunk[k], s));
            HIP_OK(hipStreamWaitEvent(c->side, c->ev_chunk[k], 0));
            ds = c->side;
        }
        if ((st = deblock_launch(c, S, ds, rows, *hb + (size_t)p0 * hb_pic, ++*ep, sched))) return st;
        p0 += n;
    }
    if (nch > 1) {
        HIP_OK(hipEventRecord(c->ev_side, c->side));
        HIP_OK(hipStreamWaitEvent(s, c->ev_side, 0));
    }
    return H264R_OK;
}

// 4:4:4 (ChromaArrayType 3): every colour plane is decoded as luma -- decode_one_component for
// PLANE_Y, PLANE_U, PLANE_V (decoder.cc:65-79) runs the luma prediction, residual and (luma-style,
// deblock.cc:422) filtering on each, with the plane's QP, levels, weights and scaling lists and the
// luma bS.  The planes never read each other, so a 4:4:4 batch runs as three 4:2:0-shaped launch
// sequences of the same kernels: pass pl's batch (k_derive444) has plane pl in the luma slots --
// records with its QP and level offset, slices with its weights, quant with its lists, DPB tables
// pointing at the references' plane pl -- and its output luma is the caller's plane pl; its own
// (empty) chroma goes to scratch.  The passes are stream-ordered and reuse one derived set.
static int run_444(h264r_ctx* c, const h264r_batch& b, hipStream_t s, int row0, int row1)
{
    const int P = b.num_pics;
    const size_t nmb = (size_t)b.width_mbs * b.height_mbs;
    const int ntab = b.ref_planes_stride ? P : 1;
    int st;
    if ((st = dev_resize(&c->d444_mbs, &c->c444_mbs, (size_t)P * nmb)) ||
        (st = dev_resize(&c->d444_slices, &c->c444_slices, (size_t)P * b.slice_stride)) ||
        (st = dev_resize(&c->d444_quant, &c->c444_quant, (size_t)P)) ||
        (st = dev_resize(&c->d444_refs, &c->c444_refs, (size_t)ntab * 3 * H264R_MAX_SLOTS)) ||
        (st = dev_resize(&c->d444_chroma, &c->c444_chroma, (size_t)P * 2 * 64 * nmb + H264R_PLANE_SLACK)))
        return st;
    const bool timing = c->timing;
    for (int pl = 0; pl < 3; ++pl) {
        hipLaunchKernelGGL(k_derive444, dim3(1024), dim3(256), 0, s, b, pl, pl, c->d444_mbs, c->d444_slices, c->d444_quant,
                           c->d444_refs, ntab, c->d_err);
        HIP_OK(hipGetLastError());
        h264r_batch d = b;
        d.mbs = c->d444_mbs; d.slices = c->d444_slices; d.quant = c->d444_quant;
        d.ref_planes = c->d444_refs;
        d.ref_planes_stride = b.ref_planes_stride ? 3 * H264R_MAX_SLOTS : 0;
        d.out_y = pl == 0 ? b.out_y : pl == 1 ? b.out_u : b.out_v;
        d.out_u = c->d444_chroma;
        d.out_v = c->d444_chroma + (size_t)P * 64 * nmb;
        if ((st = launch_all(c, d, s, row0, row1, c->sc))) return st;
    }
    if (timing) c->timed_launches -= 2;            // h264r_last_timing: per batch, its three passes together
    return H264R_OK;
}

// 4:2:2 (chroma_format_idc 2) and 4:0:0 (0): the luma plane by the 4:2:0 launch sequence (k_derive444 plane 0 --
// the records without their chroma, the DPB tables' luma planes; its chroma goes to scratch),
// then both chroma planes by k_c422_inter + k_c422_intra and, from the deblocking records that
// sequence left, k_c422_db
// (k_chroma422.hip).  Field pictures are not on this path (k_derive444 flags them).
static int run_422(h264r_ctx* c, const h264r_batch& b, hipStream_t s, int row0, int row1)
{
    const int P = b.num_pics;
    const size_t nmb = (size_t)b.width_mbs * b.height_mbs;
    const int ntab = b.ref_planes_stride ? P : 1;
    int st;
    if ((st = dev_resize(&c->d444_mbs, &c->c444_mbs, (size_t)P * nmb)) ||
        (st = dev_resize(&c->d444_slices, &c->c444_slices, (size_t)P * b.slice_stride)) ||
        (st = dev_resize(&c->d444_quant, &c->c444_quant, (size_t)P)) ||
        (st = dev_resize(&c->d444_refs, &c->c444_refs, (size_t)ntab * 3 * H264R_MAX_SLOTS)) ||
        (st = dev_resize(&c->d444_chroma, &c->c444_chroma, (size_t)P * 2 * 64 * nmb + H264R_PLANE_SLACK)))
        return st;
    // a separate-colour-plane (JV) batch on a 4:4:4 context: monochrome records, colour plane
    // jv - 1's lists, references and output plane (h264r_batch.colour_plane)
    const int jv = b.colour_plane;
    hipLaunchKernelGGL(k_derive444, dim3(1024), dim3(256), 0, s, b, 0, jv ? jv - 1 : 0, c->d444_mbs, c->d444_slices,
                       c->d444_quant, c->d444_refs, ntab, c->d_err);
    HIP_OK(hipGetLastError());
    h264r_batch d = b;
    d.colour_plane = 0;
    if (jv) d.out_y = jv == 1 ? b.out_y : jv == 2 ? b.out_u : b.out_v;
    d.mbs = c->d444_mbs; d.slices = c->d444_slices; d.quant = c->d444_quant;
    d.ref_planes = c->d444_refs;
    d.ref_planes_stride = b.ref_planes_stride ? 3 * H264R_MAX_SLOTS : 0;
    d.out_u = c->d444_chroma;
    d.out_v = c->d444_chroma + (size_t)P * 64 * nmb;
    if ((st = launch_all(c, d, s, row0, row1, c->sc))) return st;
    if (c->fmt == 0 || jv) return H264R_OK;                 // 4:0:0 / one JV plane: no chroma
    const int2 rows = make_int2(row0, row1);
    {
        Timed t(c, 0, s);
        const int64_t mbs = (int64_t)P * (row1 - row0) * b.width_mbs;
        hipLaunchKernelGGL(k_c422_inter, dim3((unsigned)((mbs + 3) / 4)), dim3(256), 0, s, b, rows, c->d_err);
        HIP_OK(hipGetLastError());
    }
    {
        Timed t(c, 1, s);
        hipLaunchKernelGGL(k_c422_intra, dim3(P), dim3(1024), 0, s, b, rows, c->d_err);
        HIP_OK(hipGetLastError());
    }
    if (!((c->debug | knobs().debug) & H264R_DBG_NO_DEBLOCK)) {
        Timed t(c, 2, s);
        hipLaunchKernelGGL(k_c422_db, dim3(P), dim3(1024), 0, s, b,
                           reinterpret_cast<const h264r::DbInfo*>(c->sc.d_dbinfo), rows, c->d_err);
        HIP_OK(hipGetLastError());
    }
    return H264R_OK;
}

// MBAFF frames (include/h264r.h H264R_MBAFF_FRAME, k_mbaff.hip): I_PCM and inter MBs in one launch,
// then the intra MBs and the loop filter each as one launch per anti-diagonal d = x + 2 y of the
// MB-pair grid (a pair's neighbours -- and the pairs its filtering modifies -- lie on earlier
// diagonals).  Whole pictures only.
static int run_mbaff(h264r_ctx* c, const h264r_batch& b, hipStream_t s, int row0, int row1)
{
    if (c->fmt != 1) return H264R_EUNSUPPORTED;
    if ((b.height_mbs & 1) || row0 != 0 || row1 != b.height_mbs) return H264R_EINVAL;
    const int P = b.num_pics, W = b.width_mbs, HP = b.height_mbs / 2, ndiag = W + 2 * (HP - 1);
    Timed whole(c, 3, s);
    if (c->timing) c->timed_launches++;
    {
        Timed t(c, 0, s);
        hipLaunchKernelGGL(k_mbaff_inter, dim3((unsigned)((size_t)P * W * b.height_mbs)), dim3(256), 0, s, b, c->d_err);
        HIP_OK(hipGetLastError());
    }
    {
        Timed t(c, 1, s);
        for (int d = 0; d < ndiag; ++d)
            hipLaunchKernelGGL(k_mbaff_intra, dim3((unsigned)(P * HP)), dim3(256), 0, s, b, d, c->d_err);
        HIP_OK(hipGetLastError());
    }
    if (!((c->debug | knobs().debug) & H264R_DBG_NO_DEBLOCK)) {
        Timed t(c, 2, s);
        for (int d = 0; d < ndiag; ++d)
            hipLaunchKernelGGL(k_mbaff_deblock, dim3((unsigned)(P * HP)), dim3(64), 0, s, b, d, c->d_err);
        HIP_OK(hipGetLastError());
    }
    return H264R_OK;
}

static int run_batch(h264r_ctx* c, const h264r_batch& b, hipStream_t s, int row0, int row1)
{
    // the scratch is shared by every launch of this context: a launch on another stream
    // than the previous one waits for it first
    if (c->last_stream && c->last_stream != s) {
        HIP_OK(hipEventRecord(c->ev_last, c->last_stream));
        HIP_OK(hipStreamWaitEvent(s, c->ev_last, 0));
    }
    c->last_stream = s;
    if (b.mbaff) return run_mbaff(c, b, s, row0, row1);
    if (b.colour_plane) {                                   // JV: one colour plane on a 4:4:4 context
        if (c->fmt != 3) return H264R_EUNSUPPORTED;
        if (b.colour_plane < 0 || b.colour_plane > 3) return H264R_EINVAL;
        return run_422(c, b, s, row0, row1);
    }
    if (c->fmt == 3) return run_444(c, b, s, row0, row1);
    if (c->fmt == 2 || c->fmt == 0) return run_422(c, b, s, row0, row1);
    return launch_all(c, b, s, row0, row1, c->sc);
}

#ifdef H264R_TRACE
void h264r_db_trace_copy(void* dst);    // k_deblock.hip / k_deblock2.hip (trace builds)
void h264r_db2_trace_copy(void* dst);
void h264r_db2y_trace_copy(void* dst);
void h264r_db2c_trace_copy(void* dst);
// H264R_TRACE_OUT=<path>: k_deblock's trace to <path>, k_deblock2's to <path>.2, the split walk's to .2y / .2c
static void dump_trace(hipStream_t s)
{
    const char* path = getenv("H264R_TRACE_OUT");
    if (!path) return;
    static std::vector<unsigned long long> buf((1 << 16) * 8);
    (void)hipStreamSynchronize(s);
    h264r_db_trace_copy(buf.data());
    if (FILE* f = fopen(path, "wb")) { fwrite(buf.data(), 8, buf.size(), f); fclose(f); }
    h264r_db2_trace_copy(buf.data());
    if (FILE* f = fopen((std::string(path) + ".2").c_str(), "wb")) { fwrite(buf.data(), 8, buf.size(), f); fclose(f); }
    h264r_db2y_trace_copy(buf.data());
    if (FILE* f = fopen((std::string(path) + ".2y").c_str(), "wb")) { fwrite(buf.data(), 8, buf.size(), f); fclose(f); }
    h264r_db2c_trace_copy(buf.data());
    if (FILE* f = fopen((std::string(path) + ".2c").c_str(), "wb")) { fwrite(buf.data(), 8, buf.size(), f); fclose(f); }
}
#endif

// ref_planes_stride: 0 (one table) or whole tables apart; per-picture tables need the caller's own
static bool stride_ok(const h264r_batch* b)
{
    return b->ref_planes_stride == 0 || (b->ref_planes_stride >= 3 * H264R_MAX_SLOTS && b->ref_planes);
}

// out_u / out_v: required, except on a 4:0:0 context, which writes no chroma (they may be NULL)
static bool chroma_out_ok(const h264r_ctx* c, const h264r_batch* b)
{
    return c->fmt == 0 || (b->out_u && b->out_v);
}

int h264r_decode_batch(h264r_ctx* c, const h264r_batch* b, void* stream)
{
    if (!c || !b || b->num_pics <= 0 || b->width_mbs <= 0 || b->height_mbs <= 0 ||
        b->width_mbs > c->max_w || b->height_mbs > c->max_h || b->slice_stride <= 0 || !b->mbs || !b->levels ||
        !b->mv || !b->ref_idx || !b->slices || !b->pics || !b->quant || !b->out_y || !chroma_out_ok(c, b) ||
        !stride_ok(b))
        return H264R_EINVAL;
    (void)hipSetDevice(c->device);
    h264r_batch bb = *b;
    if (!bb.ref_planes) bb.ref_planes = c->d_ref_planes;
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
#ifdef H264R_TRACE
    int st = run_batch(c, bb, s, 0, bb.height_mbs);
    dump_trace(s);
    return st;
#else
    return run_batch(c, bb, s, 0, bb.height_mbs);
#endif
}

int h264r_decode_batch_rows(h264r_ctx* c, const h264r_batch* b, int row0, int row1, void* stream)
{
    if (!c || !b || row0 < 0 || row1 <= row0 || row1 > b->height_mbs) return H264R_EINVAL;
    if (!b->mbs || !b->levels || !b->mv || !b->ref_idx || !b->slices || !b->pics || !b->quant || !b->out_y ||
        !chroma_out_ok(c, b) || b->num_pics <= 0 || b->width_mbs <= 0 || b->width_mbs > c->max_w ||
        b->height_mbs > c->max_h || b->slice_stride <= 0 || !stride_ok(b))
        return H264R_EINVAL;
    (void)hipSetDevice(c->device);
    h264r_batch bb = *b;
    if (!bb.ref_planes) bb.ref_planes = c->d_ref_planes;
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    return run_batch(c, bb, s, row0, row1);
}

int h264r_set_timing(h264r_ctx* c, int enable)
{
    if (!c) return H264R_EINVAL;
    c->timing = enable != 0;
    c->spans.clear();
    c->ev_used = 0;
    c->timed_launches = 0;
    return H264R_OK;
}

int h264r_check(h264r_ctx* c)
{
    if (!c) return H264R_EINVAL;
    (void)hipSetDevice(c->device);
    HIP_OK(hipStreamSynchronize(c->stream));
    if (c->last_stream) HIP_OK(hipStreamSynchronize(c->last_stream));
    if (c->side) HIP_OK(hipStreamSynchronize(c->side));
    int e = 0;
    HIP_OK(hipMemcpy(&e, c->d_err, sizeof(int), hipMemcpyDeviceToHost));
    if (e) { (void)hipMemset(c->d_err, 0, sizeof(int)); return H264R_EDEVICE; }
    return H264R_OK;
}

int h264r_set_debug(h264r_ctx* c, int flags)
{
    if (!c) return H264R_EINVAL;
    c->debug = flags;
    return H264R_OK;
}

int h264r_last_timing(h264r_ctx* c, float out[4])
{
    if (!c || !out) return H264R_EINVAL;
    if (!c->timing) return H264R_ESTATE;
    if (c->timed_launches == 0) return H264R_ESTATE;
    double sum[4] = {0, 0, 0, 0};
    for (const auto& sp : c->spans) {
        float ms = 0;
        HIP_OK(hipEventSynchronize(sp.b));
        HIP_OK(hipEventElapsedTime(&ms, sp.a, sp.b));
        sum[sp.kind] += ms;
    }
    for (int k = 0; k < 4; ++k) out[k] = (float)(sum[k] / c->timed_launches);
    c->spans.clear();
    c->ev_used = 0;
    c->timed_launches = 0;
    return H264R_OK;
}

// ------------------------------------------------------------- streaming API
int h264r_picture_begin(h264r_ctx* c, int w, int h, const h264r_pic* pic, const h264r_slice* slices,
                        const h264r_quant* quant)
{
    if (!c || !pic || !slices || !quant || w <= 0 || h <= 0 || w > c->max_w || h > c->max_h ||
        pic->num_slices <= 0 || pic->num_slices > H264R_MAX_SLICES)
        return H264R_EINVAL;
    // both staging pictures in flight: the caller collects one first (h264r_picture_wait)
    if (c->sp_pending == 2) return H264R_ESTATE;
    auto& P = c->sp[c->sp_fill];
    P.pw = w; P.ph = h;
    const size_t n = (size_t)w * h;
    P.h_mbs.assign(n, h264r_mb{});
    P.h_levels.clear();
    P.h_mv.assign(2 * 16 * n, 0);
    P.h_ref.assign(2 * 16 * n, -1);
    P.h_slices.assign(slices, slices + pic->num_slices);
    P.h_pic = *pic;
    P.h_quant = *quant;
    P.seen.assign(n, 0);
    c->in_pic = true;
    return H264R_OK;
}

int h264r_mb_submit(h264r_ctx* c, int addr, const h264r_mb* mb, const int16_t* levels, int n_levels,
                    const uint32_t* mv, const int8_t* ref_idx)
{
    if (!c) return H264R_EINVAL;
    if (!c->in_pic) return H264R_ESTATE;
    auto& P = c->sp[c->sp_fill];
    const int n = P.pw * P.ph;
    if (addr < 0 || addr >= n || !mb || n_levels < 0 || (n_levels && !levels) || !mv || !ref_idx) return H264R_EINVAL;
    if (mb->slice >= P.h_pic.num_slices) return H264R_EINVAL;
    if (mb->mb_type == H264R_SI) return H264R_EUNSUPPORTED;        // see include/h264r.h
    // lossless inter MBs: the kernels take intra_chroma_pred_mode as DC, which is what the
    // parser leaves in an inter MB (macroblock_t::init, slice_data.cc:482)
    if ((mb->flags & H264R_MBF_BYPASS) && !(mb->flags & H264R_MBF_INTRA) && mb->chroma_mode != 0) return H264R_EINVAL;
    h264r_mb m = *mb;
    // append the level block, 16-byte aligned
    while (P.h_levels.size() % 8) P.h_levels.push_back(0);
    m.coef_off = (uint32_t)P.h_levels.size();
    P.h_levels.insert(P.h_levels.end(), levels, levels + n_levels);
    P.h_mbs[addr] = m;
    const int W4 = P.pw * 4, plane = W4 * P.ph * 4, x = addr % P.pw, y = addr / P.pw;
    for (int l = 0; l < 2; ++l)
        for (int k = 0; k < 16; ++k) {
            int idx = (y * 4 + k / 4) * W4 + x * 4 + k % 4;
            P.h_mv[(size_t)l * plane + idx] = mv[l * 16 + k];
            P.h_ref[(size_t)l * plane + idx] = ref_idx[l * 16 + k];
        }
    P.seen[addr] = 1;
    return H264R_OK;
}

int h264r_picture_end_async(h264r_ctx* c, int keep_slot)
{
    if (!c) return H264R_EINVAL;
    if (!c->in_pic) return H264R_ESTATE;
    c->in_pic = false;
    auto& P = c->sp[c->sp_fill];
    for (uint8_t s : P.seen) if (!s) return H264R_ESTATE;      // every MB must be submitted
    if (keep_slot >= H264R_MAX_SLOTS) return H264R_EINVAL;
    (void)hipSetDevice(c->device);
    const size_t n = (size_t)P.pw * P.ph, ys = n * 256, cs = chroma_bytes(c, P.pw, P.ph);
    if (P.h_levels.empty()) P.h_levels.push_back(0);
    // 4:4:4: frame pictures only; a PCM MB's Cr view reads 128 entries past its block (run_444)
    if (c->fmt != 1 && P.h_pic.structure != H264R_FRAME) return H264R_EUNSUPPORTED;
    if (c->fmt != 1)                                       // SP slices are 4:2:0 only (Extended profile)
        for (const h264r_slice& sl : P.h_slices) if (sl.slice_type == H264R_SLICE_SP) return H264R_EUNSUPPORTED;
    if (c->fmt == 3) P.h_levels.insert(P.h_levels.end(), 128, 0);
    if (c->fmt == 0) P.h_levels.insert(P.h_levels.end(), 64, 0);     // the luma pass's chroma view of a PCM MB
    // every referenced slot must be loaded, with a frame of this picture's size (a field
    // picture: twice its height; its entries may name either field of a slot, include/h264r.h)
    const int fld = P.h_pic.structure == H264R_TOP_FIELD || P.h_pic.structure == H264R_BOTTOM_FIELD;
    const int mbaff = P.h_pic.structure == H264R_MBAFF_FRAME;
    if (P.h_pic.structure < H264R_FRAME || P.h_pic.structure > H264R_MBAFF_FRAME) return H264R_EINVAL;
    if (mbaff) {
        // MBAFF (include/h264r.h): 4:2:0, MB pairs, no SP slices, lossless MBs or implicit weights
        if (P.ph & 1) return H264R_EINVAL;
        for (const h264r_slice& sl : P.h_slices)
            if (sl.slice_type == H264R_SLICE_SP || sl.wp_mode == 2) return H264R_EUNSUPPORTED;
        for (const h264r_mb& m : P.h_mbs) if (m.flags & H264R_MBF_BYPASS) return H264R_EUNSUPPORTED;
        for (size_t a = 0; a < P.h_mbs.size(); a += 1) {
            const size_t top = ((a / P.pw) & ~(size_t)1) * P.pw + a % P.pw;
            if ((P.h_mbs[a].flags ^ P.h_mbs[top].flags) & H264R_MBF_FIELD) return H264R_EINVAL;   // one flag per pair
        }
        // a field MB's refIdx names field refIdx / 2 of the list
        for (size_t a = 0; a < P.h_mbs.size(); ++a) {
            const h264r_mb& m = P.h_mbs[a];
            if (m.flags & H264R_MBF_INTRA) continue;
            const int x = (int)(a % P.pw), y = (int)(a / P.pw), W4 = P.pw * 4, plane = W4 * P.ph * 4;
            const int nr = (m.flags & H264R_MBF_FIELD) ? 2 : 1;
            for (int l = 0; l < 2; ++l)
                for (int k = 0; k < 16; ++k) {
                    const int r = P.h_ref[(size_t)l * plane + (y * 4 + k / 4) * W4 + x * 4 + k % 4];
                    if (r >= nr * P.h_slices[m.slice].num_ref[l]) return H264R_EINVAL;
                }
        }
    } else if (c->fmt == 1)
        for (const h264r_mb& m : P.h_mbs) if (m.flags & H264R_MBF_FIELD) return H264R_EINVAL;
    const int frame_h = P.ph << fld;
    for (const h264r_slice& sl : P.h_slices)
        for (int l = 0; l < 2; ++l)
            for (int i = 0; i < sl.num_ref[l]; ++i) {
                const int ref = sl.ref_slot[l][i];
                const int slot = fld ? ref & ~H264R_REF_BOTTOM : ref;
                if (ref < 0 || slot >= H264R_MAX_SLOTS) return H264R_EINVAL;
                if (!c->slot[slot][0] || c->slot_w[slot] != P.pw || c->slot_h[slot] != frame_h) return H264R_ESTATE;
            }
    int st = 0;
    // the device inputs are one set, reused in stream order (dev_resize drains before it frees)
    if ((st = dev_resize(&c->d_mbs, &c->c_mbs, n)) || (st = dev_resize(&c->d_levels, &c->c_levels, P.h_levels.size())) ||
        (st = dev_resize(&c->d_mv, &c->c_mv, P.h_mv.size())) || (st = dev_resize(&c->d_ref, &c->c_ref, P.h_ref.size())) ||
        (st = dev_resize(&c->d_slices, &c->c_slices, P.h_slices.size())) || (st = dev_resize(&c->d_pic, &c->c_pic, 1)) ||
        (st = dev_resize(&c->d_quant, &c->c_quant, 1)) || (st = dev_resize(&c->d_out, &c->c_out, ys + 2 * cs)))
        return st;
    if (P.c_out < ys + 2 * cs + 16) {
        if (P.out) (void)hipHostFree(P.out);
        P.out = nullptr; P.c_out = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&P.out), ys + 2 * cs + 16) != hipSuccess) return H264R_ENOMEM;
        P.c_out = ys + 2 * cs + 16;
    }
    if (!P.done) HIP_OK(hipEventCreateWithFlags(&P.done, hipEventDisableTiming));
    hipStream_t s = c->stream;
    HIP_OK(hipMemcpyAsync(c->d_mbs, P.h_mbs.data(), n * sizeof(h264r_mb), hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(c->d_levels, P.h_levels.data(), P.h_levels.size() * 2, hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(c->d_mv, P.h_mv.data(), P.h_mv.size() * 4, hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(c->d_ref, P.h_ref.data(), P.h_ref.size(), hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(c->d_slices, P.h_slices.data(), P.h_slices.size() * sizeof(h264r_slice), hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(c->d_pic, &P.h_pic, sizeof(h264r_pic), hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(c->d_quant, &P.h_quant, sizeof(h264r_quant), hipMemcpyHostToDevice, s));
    h264r_batch b{};
    b.num_pics = 1; b.width_mbs = P.pw; b.height_mbs = P.ph; b.slice_stride = (int)P.h_slices.size();
    b.mbs = c->d_mbs; b.levels = c->d_levels; b.mv = c->d_mv; b.ref_idx = c->d_ref; b.slices = c->d_slices;
    b.pics = c->d_pic; b.quant = c->d_quant; b.ref_planes = c->d_ref_planes;
    b.out_y = c->d_out; b.out_u = c->d_out + ys; b.out_v = c->d_out + ys + cs;
    b.mbaff = mbaff;
    if ((st = run_batch(c, b, s, 0, b.height_mbs))) return st;
    if (keep_slot >= 0) {
        if ((st = ensure_slot(c, keep_slot, P.pw, frame_h))) return st;
        if (!fld) {
            HIP_OK(hipMemcpyAsync(c->slot[keep_slot][0], c->d_out, ys + 2 * cs, hipMemcpyDeviceToDevice, s));
        } else {
            // a field goes into its parity's rows of the slot's frame (the reference combines the
            // two fields of a frame with dpb_combine_field_yuv, picture.cc:578-622); the other
            // field's rows are left as they are
            const int bot = P.h_pic.structure == H264R_BOTTOM_FIELD;
            const size_t W = (size_t)P.pw * 16, Wc = W / 2;
            HIP_OK(hipMemcpy2DAsync(c->slot[keep_slot][0] + bot * W, 2 * W, c->d_out, W, W, (size_t)P.ph * 16,
                                    hipMemcpyDeviceToDevice, s));
            for (int k = 1; k < 3; ++k)
                HIP_OK(hipMemcpy2DAsync(c->slot[keep_slot][k] + bot * Wc, 2 * Wc, c->d_out + ys + (k - 1) * cs, Wc, Wc,
                                        (size_t)P.ph * 8, hipMemcpyDeviceToDevice, s));
        }
    }
    // planes and the device error word into this picture's pinned staging; the error word is
    // cleared behind it, so each picture reports its own failures
    HIP_OK(hipMemcpyAsync(P.out, c->d_out, ys + 2 * cs, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(P.out + ys + 2 * cs, c->d_err, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemsetAsync(c->d_err, 0, sizeof(int), s));
    HIP_OK(hipEventRecord(P.done, s));
    P.pending = true;
    ++c->sp_pending;
    c->sp_fill = 1 - c->sp_fill;
    return H264R_OK;
}

int h264r_picture_wait(h264r_ctx* c, uint8_t* y, uint8_t* u, uint8_t* v)
{
    if (!c) return H264R_EINVAL;
    auto& P = c->sp[c->sp_wait];
    if (!c->sp_pending || !P.pending) return H264R_ESTATE;
    (void)hipSetDevice(c->device);
    HIP_OK(hipEventSynchronize(P.done));
    P.pending = false;
    --c->sp_pending;
    c->sp_wait = 1 - c->sp_wait;
    const size_t n = (size_t)P.pw * P.ph, ys = n * 256, cs = chroma_bytes(c, P.pw, P.ph);
    if (y) memcpy(y, P.out, ys);
    if (u) memcpy(u, P.out + ys, cs);
    if (v) memcpy(v, P.out + ys + cs, cs);
    int e = 0;
    memcpy(&e, P.out + ys + 2 * cs, sizeof(int));
    return e ? H264R_EDEVICE : H264R_OK;
}

int h264r_picture_end(h264r_ctx* c, uint8_t* y, uint8_t* u, uint8_t* v, int keep_slot)
{
    if (!c) return H264R_EINVAL;
    if (c->sp_pending) return H264R_ESTATE;        // collect the asynchronous pictures first
    int st = h264r_picture_end_async(c, keep_slot);
    if (st) return st;
    return h264r_picture_wait(c, y, u, v);
}

}  // extern "C"

#ifdef H264R_TRACE_INTRA
// Diagnostic build only: copy the per-MB timing trace of k_intra_levels to the host.
extern "C" __global__ void k_intra_trace_dump(unsigned long long* out, unsigned* n);
extern "C" int h264r_trace_intra_dump(unsigned long long* out_host, unsigned* n_host)
{
    unsigned long long* d = nullptr;
    unsigned* dn = nullptr;
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMalloc(&d, (size_t(1) << 20) * 32));
    HIP_OK(hipMalloc(&dn, 4));
    hipLaunchKernelGGL(k_intra_trace_dump, dim3(256), dim3(256), 0, nullptr, d, dn);
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(n_host, dn, 4, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(out_host, d, (size_t)*n_host * 32, hipMemcpyDeviceToHost));
    (void)hipFree(d); (void)hipFree(dn);
    return 0;
}
#endif
